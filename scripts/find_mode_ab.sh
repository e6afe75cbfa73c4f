#!/bin/bash
# Dev: the closed step under MIOpen find modes (default / NORMAL / HYBRID) for the ConvVAE convolutions.
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for m in default 1 3; do
  t0=$(date +%s.%N)
  if [ $m = default ]; then E=""; else E="MIOPEN_FIND_MODE=$m"; fi
  timeout -k 10 300 env $E python3 bench.py --regime closed --steps 20 --warmup 3 --no-cpu-baseline --no-c2 > gpurun_out/fm_$m.json 2> gpurun_out/fm_$m.err || { tail -5 gpurun_out/fm_$m.err; exit 1; }
  t1=$(date +%s.%N)
  python3 -c "
import json; d=json.load(open('gpurun_out/fm_$m.json')); print('mode $m round $r', round(d['ms_per_step'],3), 'wall', round($t1-$t0,1), 's')"
done
done
