#!/bin/bash
# Regime A alone with its data-parallel step through a world-1 RCCL group (bench.py's regime_a.dp_world1_rccl).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/ra_dp1; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --regime hensman --no-cpu-baseline --dp-world1 > $OUT/ra.json 2> $OUT/ra.err || { tail -20 $OUT/ra.err; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/ra.json'))
print('regime A', round(d['ms_per_step'], 3), 'ms; dp world-1 RCCL', d.get('dp_world1_rccl'))"
