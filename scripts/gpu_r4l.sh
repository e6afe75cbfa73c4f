#!/bin/bash
# Round-4: Regime A (graphed Hensman step) kernel stats + one-step timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4l}
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --regime hensman --h-steps 200 --warmup 5 --no-cpu-baseline > $OUT/h.json 2> $OUT/h.err || { tail -5 $OUT/h.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/h.json').read().strip().splitlines()[-1]); print('hensman', round(d['ms_per_step'],4), 'ms')"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/hprof -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime hensman --h-steps 50 --warmup 5 --no-cpu-baseline > $OUT/hprof.json 2> $OUT/hprof.err || { tail -5 $OUT/hprof.err; exit 1; }
python3 - $OUT/hprof/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = 57  # warm-up (5) + graph capture warm-up (~2) + 50 timed
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time {tot/1e3:.0f} us over the run; per ~step {tot/steps/1e3:.1f} us")
for r in rows[:40]:
    print(f"{float(r['TotalDurationNs'])/steps/1e3:8.1f} us/step {int(r['Calls'])/steps:6.2f}/step avg {float(r['AverageNs'])/1e3:8.1f}  {r['Name'][:100]}")
PY
python3 $ROOT/scripts/timeline.py $(find $OUT/hprof -name '*kernel_trace.csv' | head -1) multi_tensor_apply > $OUT/h_timeline.txt 2>&1; head -3 $OUT/h_timeline.txt
find $OUT/hprof -name '*kernel_trace.csv' -delete
