#!/bin/bash
# Dev: same-box A/B of two bench argument sets for the closed step: "a" = $A_ARGS, "b" = $B_ARGS, ROUNDS alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/args_ab; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in a b; do
    if [ $v = a ]; then X="$A_ARGS"; else X="$B_ARGS"; fi
    timeout -k 10 300 python3 bench.py --regime closed --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline --no-c2 $X \
      > $OUT/$v$r.json 2> $OUT/$v$r.err || { tail -5 $OUT/$v$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/$v$r.json'))
print('$v round $r: ms/step', round(d['ms_per_step'], 3), {k: round(v, 3) for k, v in d['phase_ms_per_step'].items()})"
  done
done
