#!/bin/bash
# Round 4: one graphed Hensman step's kernel timeline after the glue fusion (Regime A critical path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4q}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/h -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime hensman --steps 1 --warmup 1 --h-steps 30 --no-cpu-baseline --no-phase-timing \
  --no-c2 > $OUT/h.json 2> $OUT/h.err || { tail -5 $OUT/h.err; exit 1; }
python3 $ROOT/scripts/timeline.py $OUT/h/run_kernel_trace.csv hn_reduce > $OUT/hensman_timeline.txt
rm -f $OUT/h/run_kernel_trace.csv
head -3 $OUT/hensman_timeline.txt
