#!/bin/bash
# Dev: build the HIP library with extra compile definitions ($DEFS, e.g. "-DLVAE_C16NS=4") into
# build_ab/liblvae_hip.so, for the same-box A/B of scripts/step_ab.sh.
cd "$(dirname "$0")/.." || exit 2
mkdir -p build_ab/obj
pids=()
for s in longitudinal-vae_amd/csrc/*.hip longitudinal-vae_amd/csrc/*.cpp; do
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-pass-failed $DEFS -I include -c "$s" \
    -o build_ab/obj/$(basename "$s").o & pids+=($!)
done
for p in "${pids[@]}"; do wait $p || exit 1; done
hipcc --offload-arch=gfx950 -shared -fPIC -o build_ab/liblvae_hip.so build_ab/obj/*.o
