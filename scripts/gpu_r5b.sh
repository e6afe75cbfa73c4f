#!/bin/bash
# Round 5: the histogram Gram adjoint (kl_gram_bwd_hist_kernel) -- parity (the Regime B KL tests, the gloo world-2
# CUDA test) and a same-box A/B of the adjoint alone against the table kernel (LVAE_GRAM_HIST=0), rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r5b; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PYT tests/test_gpu_regime_b.py tests/test_gpu_rccl.py -k "kl_closed or gloo or prefactor" -s \
  > $OUT/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |Error" $OUT/pytest.log | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $ROOT/scripts/gram_micro.py 2 > $OUT/warm.log 2>&1 || exit $?
run() {
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ab_$1 -o run --output-format csv -- \
    python3 $ROOT/scripts/gram_micro.py 5 > $OUT/micro_$1.log 2>&1 || exit $?
  rm -f $OUT/ab_$1/*kernel_trace.csv
}
run hist
LVAE_GRAM_HIST=0 run tab
run hist2
LVAE_GRAM_HIST=0 run tab2
grep -h "hyper-grads" $OUT/micro_*.log
for d in hist tab hist2 tab2; do grep -h "kl_gram_bwd" $OUT/ab_$d/run_kernel_stats.csv | awk -F, -v d=$d '{print d, $1, $2, $4}' ; done
