#!/bin/bash
# Round 4: the fused glue launches (glue.hip) -- the -m gpu suite, then the closed step at the headline and
# at the 8-GPU rank share, and the graphed Hensman step (LVAE_GLUE=0 would need a rebuild: the A/B is against
# the committed r4 numbers of the same box type).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4p}
mkdir -p $OUT
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider --maxfail=5 ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
[ $rc -le 1 ] || exit $rc
for v in "h:--regime closed" "s8:--regime closed --rank-share 8" "h2:--regime closed" "s8b:--regime closed --rank-share 8"; do
  name=${v%%:*}; args=${v#*:}
  echo "[$(date +%T)] bench $name"
  timeout -k 10 300 python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -20 $OUT/b_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$name.json')); print('$name', round(d['ms_per_step'],3), 'ms', d.get('clock', {}).get('gfx_mhz_median'))"
done
echo "[$(date +%T)] hensman"
timeout -k 10 300 python3 bench.py --regime hensman --steps 1 --warmup 1 --h-steps 100 --no-cpu-baseline --no-c2 > $OUT/b_hens.json 2> $OUT/b_hens.err || { tail -20 $OUT/b_hens.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_hens.json')); a=d.get('regime_a', d); print('hensman', a.get('ms_per_step'))"
