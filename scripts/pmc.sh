#!/bin/bash
# HBM traffic of the Regime B step's kernels: separate rocprofv3 PMC passes for FETCH_SIZE and
# WRITE_SIZE (MI355X_MICROARCH.md: TCC slots do not fit both), kernel trace only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -d $OUT/$c -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-phase-timing > $OUT/$c.json 2> $OUT/$c.err || exit $?
done
python3 $ROOT/scripts/pmc_summary.py $OUT > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
rm -rf $OUT/FETCH_SIZE $OUT/WRITE_SIZE
