#!/bin/bash
# Dev: same-box A/B of the closed step's ConvVAE stream priority (bench.py --vae-stream-priority 0 / -1),
# interleaved rounds; then a one-step kernel timeline at the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2; do
  for p in 0 -1; do
    timeout -k 10 300 python3 bench.py --regime closed --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-c2 \
      --vae-stream-priority $p $BENCH_ARGS > $OUT/prio_$p$r.json 2> $OUT/prio_$p$r.err || { tail -5 $OUT/prio_$p$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/prio_$p$r.json'))
print('priority $p round $r: ms/step', round(d['ms_per_step'], 3), {k: round(v, 3) for k, v in d['phase_ms_per_step'].items()})"
  done
done
NAME=prio bash scripts/trace_step.sh $BENCH_ARGS
