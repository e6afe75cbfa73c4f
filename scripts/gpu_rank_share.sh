#!/bin/bash
# One rank's share of the W-GPU latent-sharded closed step, timed on one GPU (bench.py --rank-share W: L/W dims, N/W
# images, collectives replaced by local stand-ins), W in $WS, ROUNDS interleaved; then the one-GPU step for reference.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/share; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for w in ${WS:-1 2 4 8}; do
    A="--rank-share $w"; [ $w = 1 ] && A=""
    timeout -k 10 300 python3 bench.py --regime closed --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline --no-c2 $A \
      > $OUT/w$w-$r.json 2> $OUT/w$w-$r.err || { tail -5 $OUT/w$w-$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/w$w-$r.json'))
print('W=$w round $r: ms/step', round(d['ms_per_step'], 3), 'potrf', round(d['phase_ms_per_step'].get('potrf', 0), 3))"
  done
done
