#!/bin/bash
# Dev: same-box A/B of the closed step timed eagerly vs as one HIP graph (bench.py default / --graph).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2; do
  for m in eager graph; do
    flag=""; [ $m = graph ] && flag="--graph"
    timeout -k 10 300 python3 bench.py --regime closed --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-c2 \
      $flag $BENCH_ARGS > $OUT/graph_ab_$m$r.json 2> $OUT/graph_ab_$m$r.err || { tail -5 $OUT/graph_ab_$m$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/graph_ab_$m$r.json'))
print('$m round $r: ms/step', round(d['ms_per_step'], 3), 'roofline', round(d['roofline']['frac'], 3), {k: round(v, 3) for k, v in d['phase_ms_per_step'].items()})"
  done
done
