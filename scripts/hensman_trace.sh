#!/bin/bash
# rocprofv3 kernel trace of the graphed Hensman bench step; per-step kernel list (hensman_trace.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-htrace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime hensman --steps 1 --warmup 1 --h-steps 30 --no-cpu-baseline --no-phase-timing \
  --no-c2 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 $ROOT/scripts/hensman_trace.py $OUT/run_kernel_trace.csv | tee $OUT/steps.txt
rm -f $OUT/run_kernel_trace.csv
