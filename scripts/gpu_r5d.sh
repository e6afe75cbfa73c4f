#!/bin/bash
# Round 5: the binned hyper-gradient route (kl_hyper.hip) -- its tests, the Regime B suite, then the KL micro
# (fwd + bwd alone) under rocprofv3 with the route on and off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r5c; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PYT tests/test_gpu_kl_hyper.py -x -s > $OUT/hyper.log 2>&1; rc=$?
grep -E "passed|failed|rel err|route raw" $OUT/hyper.log | tail -20
[ $rc -eq 0 ] || { grep -E "^E |Error" $OUT/hyper.log | head -30; exit $rc; }
[ -n "$FULL" ] && { timeout -k 10 600 $PYT tests/test_gpu_regime_b.py tests/test_gpu_rccl.py tests/test_gpu_linalg.py > $OUT/regb.log 2>&1; rc=$?; } || rc=0
grep -E "passed|failed" $OUT/regb.log | tail -3
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/regb.log | head -30; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $ROOT/scripts/gram_micro.py 2 > $OUT/warm.log 2>&1 || exit $?
run() {
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ab_$1 -o run --output-format csv -- \
    python3 $ROOT/scripts/gram_micro.py 5 > $OUT/micro_$1.log 2>&1 || exit $?
  rm -f $OUT/ab_$1/*kernel_trace.csv
}
run hb
LVAE_KL_HYPER=0 run gemm
grep -h "hyper-grads" $OUT/micro_*.log
cd $ROOT
for d in hb gemm; do echo "== $d"; python3 scripts/kstats.py $OUT/ab_$d/run_kernel_stats.csv 14 1; done
