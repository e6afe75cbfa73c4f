#!/bin/bash
# Round-4: inverse-only A/B of the schedule switches (scripts/inv_ab.py), then share8 steps (60 each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4e}
mkdir -p $OUT
inv() { env "$@" timeout -k 10 120 python3 scripts/inv_ab.py 2>/dev/null | grep median || { echo "inv failed: $*"; exit 1; }; }
for Lv in 2 4; do
  inv L=$Lv LVAE_CI_PIPE=0 LVAE_PIVOT_SPLIT=0
  inv L=$Lv LVAE_CI_PIPE=0 LVAE_PIVOT_SPLIT=1
  inv L=$Lv LVAE_CI_PIPE_LAUUM=0 LVAE_CI_PAIR=0
  inv L=$Lv LVAE_CI_PAIR=0
  inv L=$Lv LVAE_CI_PAIR=1
  inv L=$Lv LVAE_CI_PIPE_LAUUM=0 LVAE_CI_PAIR=1
done
inv L=16 LVAE_PIVOT_SPLIT=0
inv L=16 LVAE_PIVOT_SPLIT=1
bench() {  # name env... -- args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 bench.py "$@" --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -20 $OUT/b_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
}
for r in 1 2; do
  bench s8_p0_$r LVAE_CI_PIPE=0 -- --regime closed --rank-share 8 || exit 1
  bench s8_p1_$r LVAE_CI_PIPE_LAUUM=0 LVAE_CI_PAIR=0 -- --regime closed --rank-share 8 || exit 1
  bench s8_p2_$r LVAE_CI_PAIR=0 -- --regime closed --rank-share 8 || exit 1
done
