#!/bin/bash
# Round 4: the fp64 diag(K^-1) refinement (kl_refine.hip) -- the -m gpu suite (its printed gate per dim),
# then the default closed bench and the rank-share-4 bench (no dim of the bench's step may be flagged).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4n}
mkdir -p $OUT
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider --maxfail=5 ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
[ $rc -le 1 ] || exit $rc
for v in "h:--regime closed" "s4:--regime closed --rank-share 4"; do
  name=${v%%:*}; args=${v#*:}
  echo "[$(date +%T)] bench $name"
  timeout -k 10 300 python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -20 $OUT/b_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$name.json')); print('$name', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
done
