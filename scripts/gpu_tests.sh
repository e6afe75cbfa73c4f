#!/bin/bash
# GPU parity tests (all, or -k "$K"), then optionally a short Regime B bench without the CPU leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out
mkdir -p $OUT
echo "[$(date +%T)] pytest -m gpu ${K:+-k "$K"}"
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu ${PYTEST_X:--x} -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|rel err|errors|passed|failed|Error" $OUT/pytest_gpu.log | tail -60
[ $rc -eq 0 ] || exit $rc
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
echo "[$(date +%T)] bench"
timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err
exit $rc
