#!/bin/bash
# Dev: rocprofv3 kernel trace of a few closed steps (args: bench.py args), one step's timeline printed
# by scripts/timeline.py into gpurun_out/timeline_$NAME.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
NAME=${NAME:-h}
OUT=$ROOT/gpurun_out/trace_$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed "$@" --steps 4 --warmup 2 --no-cpu-baseline --no-phase-timing --no-c2 \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 $ROOT/scripts/timeline.py $(find $OUT -name '*kernel_trace.csv' | head -1) > $ROOT/gpurun_out/timeline_$NAME.txt
find $OUT -name '*kernel_trace.csv' -delete
head -3 $ROOT/gpurun_out/timeline_$NAME.txt
