#!/bin/bash
# Timing of the binned route's slab pass with parts skipped (LVAE_HB_DBG bits: 1 H, 2 near runs, 4 tr S):
# the KL micro under rocprofv3 per mask; prints the hb kernels' averages.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/hbdbg; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $ROOT/scripts/gram_micro.py 2 > $OUT/warm.log 2>&1 || exit $?
for m in ${MASKS:-0 1 2 4 7 8 16 32 63}; do
  LVAE_HB_DBG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/m$m -o run --output-format csv -- \
    python3 $ROOT/scripts/gram_micro.py 3 > $OUT/micro_$m.log 2>&1 || exit $?
  rm -f $OUT/m$m/*kernel_trace.csv
  echo "== mask $m"; python3 $ROOT/scripts/kstats.py $OUT/m$m/run_kernel_stats.csv 40 1 | grep "hb_"
done
