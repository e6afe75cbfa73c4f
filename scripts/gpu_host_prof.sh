#!/bin/bash
# Host-side (Python) profile of the timed steps of the W-rank share (bench.py LVAE_BENCH_CPROFILE): top functions.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/hostprof; mkdir -p $OUT
W=${W:-8}
A="--rank-share $W"; [ $W = 1 ] && A=""
LVAE_BENCH_CPROFILE=$OUT/share$W.prof timeout -k 10 300 python3 bench.py --regime closed --steps 200 --warmup 5 \
  --no-cpu-baseline --no-c2 $A --no-phase-timing > $OUT/share$W.json 2> $OUT/share$W.err || { tail -5 $OUT/share$W.err; exit 1; }
python3 -c "
import pstats
s = pstats.Stats('$OUT/share$W.prof'); s.sort_stats('tottime').print_stats(50)
s.sort_stats('cumulative').print_stats(70)" > $OUT/share${W}_top.txt
python3 -c "import json; print(json.load(open('$OUT/share$W.json'))['ms_per_step'])"
