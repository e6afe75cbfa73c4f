#!/bin/bash
# Gram adjoint chunk tables: 3 / 2 waves per SIMD (build_wpe3 / build_wpe2, LVAE_TAB_G workgroups)
# against the previous kernel (build_ab), same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r4y2; mkdir -p $OUT
SO=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so
cp $SO /tmp/new.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $ROOT/scripts/gram_micro.py 2 > $OUT/warm.log 2>&1 || exit $?
run() {
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ab_$1 -o run --output-format csv -- \
    python3 $ROOT/scripts/gram_micro.py 5 > $OUT/micro_$1.log 2>&1 || exit $?
  rm -f $OUT/ab_$1/*kernel_trace.csv
}
cp $ROOT/build_ab/liblvae_hip.so $SO; run old
cp $ROOT/build_wpe3/liblvae_hip.so $SO; run w3
cp $ROOT/build_wpe2/liblvae_hip.so $SO; run w2
LVAE_TAB_G=1024 run w2g1024
LVAE_TAB_G=512 run w2g512
cp $ROOT/build_ab/liblvae_hip.so $SO; run old2
cp $ROOT/build_wpe3/liblvae_hip.so $SO; run w3b
cp /tmp/new.so $SO
grep -h "hyper-grads" $OUT/micro_*.log
