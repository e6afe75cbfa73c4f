#!/bin/bash
# Kernel timeline of the batched sweep alone (rocprofv3 kernel trace of scripts/sweep_micro.py):
# per pass, start / end of pivot, prep0, prepW, U1, U2 relative to the sweep's first kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TL_NAME:-timeline}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- \
  python3 $ROOT/scripts/sweep_micro.py ${TL_N:-4096} ${TL_L:-16} 4 > $OUT/micro.log 2>&1 || { cat $OUT/micro.log; exit 1; }
cat $OUT/micro.log
python3 $ROOT/scripts/sweep_timeline.py $OUT/run_kernel_trace.csv | tee $OUT/timeline.txt
rm -f $OUT/run_kernel_trace.csv
