#!/bin/bash
# Dev A/B: the W = 8 rank share (bench.py --rank-share 8) with the binned hyper route on / off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/share_ab; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --regime closed --rank-share 8 --steps 5 --warmup 3 --no-cpu-baseline --no-c2 > $OUT/warm.json 2> $OUT/warm.err || exit 1
for r in 1 2; do
  for v in 1 0; do
    LVAE_KL_HYPER=$v timeout -k 10 300 python3 bench.py --regime closed --rank-share 8 --steps 40 --warmup 5 --no-cpu-baseline --no-c2 \
      > $OUT/h$v.$r.json 2> $OUT/h$v.$r.err || { tail -5 $OUT/h$v.$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/h$v.$r.json'))
print('hyper $v round $r: ms/step', round(d['ms_per_step'], 3), {k: round(x, 3) for k, x in d['phase_ms_per_step'].items()})"
  done
done
