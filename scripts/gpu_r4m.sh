#!/bin/bash
# Round-4: lookahead split of the trailing update (LVAE_CI_LOOKAHEAD) -- -m gpu, inverse-only, headline / share A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4m}
mkdir -p $OUT
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider --maxfail=5 \
  > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
[ $rc -le 1 ] || exit $rc
inv() { env "$@" timeout -k 10 120 python3 scripts/inv_ab.py 2>/dev/null | grep median || { echo "inv failed: $*"; exit 1; }; }
for Lv in 16 8 4; do
  inv L=$Lv LVAE_CI_LOOKAHEAD=0
  inv L=$Lv LVAE_CI_LOOKAHEAD=1
done
inv L=4 NP=16384 REPS=5 LVAE_CI_LOOKAHEAD=0
inv L=4 NP=16384 REPS=5 LVAE_CI_LOOKAHEAD=1
bench() {  # name env... -- args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 bench.py "$@" --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -20 $OUT/b_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
}
for r in 1 2; do
  bench h_la0_$r LVAE_CI_LOOKAHEAD=0 -- --regime closed || exit 1
  bench h_la1_$r LVAE_CI_LOOKAHEAD=1 -- --regime closed || exit 1
  bench s4_la0_$r LVAE_CI_LOOKAHEAD=0 -- --regime closed --rank-share 4 || exit 1
  bench s4_la1_$r LVAE_CI_LOOKAHEAD=1 -- --regime closed --rank-share 4 || exit 1
done
