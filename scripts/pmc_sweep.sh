#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over the Regime B bench step,
# restricted to kernels matching $RE; summary via pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PMC_NAME:-pmc_sweep}
RE=${RE:-sw_|syrk}
mkdir -p $OUT
timeout -k 10 300 python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-phase-timing > /dev/null 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex "$RE" -d $OUT/p$i -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-phase-timing > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i ($c) rc=$?"; tail -5 $OUT/p$i.err; exit 1; }
done
python3 $ROOT/scripts/pmc_summary.py $OUT > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
for i in 1 2 3 4; do rm -f $OUT/p$i/*kernel_trace.csv; done
find $OUT -name "*counter_collection.csv" -size +20M -delete
