#!/bin/bash
# Quick GPU iteration: selected parity tests (-k $K) then the Regime B bench (phase timing on).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out
mkdir -p $OUT
echo "[$(date +%T)] pytest -k '${K:-sweep or kl_closed}'"
timeout -k 10 300 python -u -m pytest tests/test_gpu_regime_b.py -m gpu -x -v -s --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "${K:-sweep or kl_closed}" > $OUT/iter_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|rel err|passed|failed" $OUT/iter_pytest.log | tail -40
[ $rc -eq 0 ] || exit $rc
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
echo "[$(date +%T)] bench"
timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline $BENCH_ARGS > $OUT/iter_bench.json 2> $OUT/iter_bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/iter_bench.json; tail -3 $OUT/iter_bench.err
exit $rc
