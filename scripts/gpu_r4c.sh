#!/bin/bash
# Round-4: the split pivot (kCiPvG workgroups per pending pivot) -- -m gpu suite, then share8 / headline /
# L=2 with LVAE_PIVOT_SPLIT=0 / 1, and the pivot phase stamps of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
N=${PROF_NAME:-r4c}
OUT=$ROOT/gpurun_out/$N
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
    -p no:cacheprovider --maxfail=5 ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
  [ $rc -le 1 ] || exit $rc
fi
bench() {  # name env... -- args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 bench.py "$@" --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -20 $OUT/b_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
}
for r in 1 2; do
  bench share8_s0_$r LVAE_PIVOT_SPLIT=0 -- --regime closed --rank-share 8 || exit 1
  bench share8_s1_$r LVAE_PIVOT_SPLIT=1 -- --regime closed --rank-share 8 || exit 1
  bench head_s0_$r LVAE_PIVOT_SPLIT=0 -- --regime closed || exit 1
  bench head_s1_$r LVAE_PIVOT_SPLIT=1 -- --regime closed || exit 1
done
for v in 0 1; do
  echo "[$(date +%T)] pivot_prof split=$v"
  LVAE_PIVOT_SPLIT=$v LS=2,16 timeout -k 10 120 python3 scripts/pivot_prof.py > $OUT/pivot_prof_s$v.txt 2>&1 || { tail -5 $OUT/pivot_prof_s$v.txt; exit 1; }
  grep -E "^L=|^  (1|2|8|15) " $OUT/pivot_prof_s$v.txt
done
