#!/bin/bash
# Round-4: the rank-share step after the hyper-backward reorder (share 8 / 4 / 2), the headline, a timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4i}
mkdir -p $OUT
bench() {  # name env... -- args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 bench.py "$@" --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -20 $OUT/b_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
}
for r in 1 2; do
  bench s8_$r X=1 -- --regime closed --rank-share 8 || exit 1
  bench s8np_$r LVAE_CI_PIPE=0 -- --regime closed --rank-share 8 || exit 1
done
bench s4 X=1 -- --regime closed --rank-share 4 || exit 1
bench s4np LVAE_CI_PIPE=0 -- --regime closed --rank-share 4 || exit 1
bench s2 X=1 -- --regime closed --rank-share 2 || exit 1
bench s1 X=1 -- --regime closed --sharded-world1 || exit 1
bench h X=1 -- --regime closed || exit 1
NAME=s8_r bash scripts/trace_step.sh --rank-share 8 || exit 1
