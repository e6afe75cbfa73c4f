#!/bin/bash
# Dev A/B: the slab pass's fp64 fold interval (LVAE_HB_FOLD builds in build_f8/, build_f16/ vs the tree's 4):
# the binned-route tests' errors with each library, then the slab pass's time (rocprofv3 over the KL micro).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/fold_ab; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
for f in ${FOLDS:-4 8 16}; do
  if [ $f = ${TREE_FOLD:-4} ]; then LIB=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so; else LIB=$ROOT/build_f$f/liblvae_hip.so; fi
  LVAE_LIB=$LIB timeout -k 10 300 $PYT tests/test_gpu_kl_hyper.py -x -s > $OUT/hyper_$f.log 2>&1 || { tail -20 $OUT/hyper_$f.log; exit 1; }
  echo "== fold $f"; grep -E "passed|rel err|routes agree|raw gradients" $OUT/hyper_$f.log | tail -12
  (cd /tmp && export TMPDIR=/tmp && LVAE_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/m$f -o run \
    --output-format csv -- python3 $ROOT/scripts/gram_micro.py 3 > $OUT/micro_$f.log 2>&1) || exit 1
  rm -f $OUT/m$f/*kernel_trace.csv
  python3 $ROOT/scripts/kstats.py $OUT/m$f/run_kernel_stats.csv 40 1 | grep "hb_slab"
done
