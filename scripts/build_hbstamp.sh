#!/bin/bash
# Diagnostic library: kl_hyper.hip with LVAE_HB_STAMP (per-section cycle stamps), the rest as built in-tree.
# Output build_diag/liblvae_hip.so; load it with LVAE_LIB=<path>.
set -e
cd "$(dirname "$0")/.."
mkdir -p build_diag
C=longitudinal-vae_amd/csrc
hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-pass-failed -DLVAE_HB_STAMP -I include -c $C/kl_hyper.hip -o build_diag/kl_hyper.o
objs=$(ls $C/*.hip.o $C/*.cpp.o 2>/dev/null | grep -v kl_hyper)
hipcc --offload-arch=gfx950 -shared -fPIC -o build_diag/liblvae_hip.so $objs build_diag/kl_hyper.o
