#!/bin/bash
# W-rank share (bench.py --rank-share W) of the round-5 tree (variants/r5tree, a git worktree of the round-5 end
# commit, built in place) against this tree, alternated on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$PWD; OUT=$ROOT/gpurun_out/r5r6; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-3}); do
  for t in ${ORDER:-r5 r6}; do
    D=$ROOT; [ $t = r5 ] && D=$ROOT/variants/r5tree
    (cd $D && timeout -k 10 300 python3 bench.py --regime closed --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline --no-c2 \
      --rank-share ${W:-8} > $OUT/$t-$r.json 2> $OUT/$t-$r.err) || { tail -5 $OUT/$t-$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/$t-$r.json'))
print('$t round $r: ms/step', round(d['ms_per_step'], 3), {k: round(v, 3) for k, v in d['phase_ms_per_step'].items()})"
  done
done
