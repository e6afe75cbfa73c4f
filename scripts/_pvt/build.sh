#!/bin/bash
# Diagnostic build of the HIP library with the sw_pivot_kernel phase probes (-DLVAE_PV_TIMING).
set -e
cd "$(dirname "$0")/../../longitudinal-vae_amd/csrc"
objs=()
for f in *.hip *.cpp; do
  o=/tmp/pvt_${f//./_}.o
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-pass-failed -I ../../include -DLVAE_PV_TIMING -c "$f" -o "$o"
  objs+=("$o")
done
hipcc --offload-arch=gfx950 -shared -fPIC -o ../../scripts/_pvt/liblvae_pvt.so "${objs[@]}"
