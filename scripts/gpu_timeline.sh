#!/bin/bash
# One closed bench step's kernel timeline per queue (rocprofv3 --kernel-trace; scripts/timeline.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/${NAME:-tl}; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --regime closed --steps 5 --warmup 3 --no-cpu-baseline --no-c2 ${BENCH_ARGS} > $OUT/warm.json 2> $OUT/warm.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --steps 8 --warmup 3 --no-cpu-baseline --no-c2 --no-phase-timing ${BENCH_ARGS} > $OUT/tr.json 2> $OUT/tr.err || exit $?
python3 $ROOT/scripts/timeline.py $(ls $OUT/tr/*kernel_trace.csv | head -1) ${MARK:-gram_sq_fill_tab} > $OUT/timeline.txt
gzip -f $OUT/tr/*kernel_trace.csv
cat $OUT/timeline.txt | head -150
