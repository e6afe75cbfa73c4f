#!/bin/bash
# Round 4: one headline closed step's kernel timeline (all streams), after a warm-up run for MIOpen's find DB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4s}
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --regime closed --steps 3 --warmup 2 --no-cpu-baseline --no-c2 > /dev/null 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --steps 4 --warmup 2 --no-cpu-baseline --no-c2 --no-phase-timing \
  > $OUT/t.json 2> $OUT/t.err || { tail -5 $OUT/t.err; exit 1; }
python3 $ROOT/scripts/timeline.py $OUT/t/run_kernel_trace.csv > $OUT/closed_timeline.txt
rm -f $OUT/t/run_kernel_trace.csv
head -3 $OUT/closed_timeline.txt
