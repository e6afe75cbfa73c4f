#!/bin/bash
# Dev GPU call: the S-GEMM core A/B (scripts/gemm_ab.py), then the exact-KL parity tests, then a short bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out
mkdir -p $OUT
if [ -n "$VARIANTS" ]; then
  echo "[$(date +%T)] gemm A/B $VARIANTS"
  timeout -k 10 300 python -u scripts/gemm_ab.py > $OUT/gemm_ab.txt 2>&1 || { cat $OUT/gemm_ab.txt; exit 1; }
  cat $OUT/gemm_ab.txt
fi
echo "[$(date +%T)] pytest -k ${K:-kl_closed}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${K:-kl_closed}" > $OUT/pytest_ab.log 2>&1
rc=$?; tail -5 $OUT/pytest_ab.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_ab.log | head -30; exit $rc; }
echo "[$(date +%T)] bench"
timeout -k 10 300 python bench.py --regime closed --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-c2 $BENCH_ARGS \
  > $OUT/bench_ab.json 2> $OUT/bench_ab.err || { tail -20 $OUT/bench_ab.err; exit 1; }
python -c "
import json; d = json.load(open('$OUT/bench_ab.json'))
print('ms/step', round(d['ms_per_step'], 3), {k: round(v, 3) for k, v in d['phase_ms_per_step'].items()}, 'roofline', round(d['roofline']['frac'], 3))"
