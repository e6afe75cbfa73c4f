#!/bin/bash
# Round 4: the -m gpu suite (incl. the C5-size forced refinement) and the graphed Hensman bench (3 runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4w}
mkdir -p $OUT
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider --maxfail=5 > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -8
[ $rc -le 1 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --regime hensman --steps 1 --warmup 1 --h-steps 100 --no-cpu-baseline --no-c2 > $OUT/b_hens_$r.json 2> $OUT/b_hens_$r.err || { tail -20 $OUT/b_hens_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_hens_$r.json')); print('hensman', d.get('ms_per_step'))"
done
