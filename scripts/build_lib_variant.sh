#!/bin/bash
# Dev: a variant of the HIP library with extra compile definitions for the listed sources: SRCS="kl_hyper.hip"
# DEFS="-DLVAE_HB_DEPTH=4" NAME=d4 -> variants/d4/liblvae_hip.so (the tree's other objects reused; build() first).
# Selected at run time by LVAE_LIB=variants/<NAME>/liblvae_hip.so (scripts/lib_ab.sh).
cd "$(dirname "$0")/.." || exit 2
C=longitudinal-vae_amd/csrc; V=variants/$NAME; mkdir -p $V/obj
objs=()
for o in $C/*.o; do
  b=$(basename $o .o)
  if [[ " $SRCS " == *" $b "* ]]; then
    hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-pass-failed $DEFS -I include -c $C/$b -o $V/obj/$b.o || exit 1
    objs+=($V/obj/$b.o)
  else
    objs+=($o)
  fi
done
hipcc --offload-arch=gfx950 -shared -fPIC -o $V/liblvae_hip.so "${objs[@]}" && rm -rf $V/obj && echo "$V/liblvae_hip.so"
