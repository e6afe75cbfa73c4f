#!/bin/bash
# Round-3 PMC passes over the closed step (bench.py --regime closed, 2 steps + 1 warm-up, kernel trace
# only, one counter group per run), summarised per kernel: per dispatch (mean) and per step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PMC_NAME:-pmc_r3}
mkdir -p $OUT
# warm MIOpen's find database first
timeout -k 10 300 python3 $ROOT/bench.py --regime closed --steps 1 --warmup 1 --no-cpu-baseline --no-phase-timing --no-c2 \
  > /dev/null 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
PASSES=${PASSES:-"FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"}
IFS=';' read -ra P <<< "$PASSES"
i=0
for c in "${P[@]}"; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $c"
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $OUT/p$i -o run --output-format csv -- \
    python3 $ROOT/bench.py --regime closed ${PMC_ARGS} --steps 2 --warmup 1 --no-cpu-baseline --no-phase-timing --no-c2 \
    > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -5 $OUT/p$i.err; exit 1; }
done
PMC_STEPS=3 PMC_KERNELS=${PMC_KERNELS:-"syrk,ci_,kl_,gram_"} python3 $ROOT/scripts/pmc_summary.py $OUT > $OUT/pmc_summary.txt
cat $OUT/pmc_summary.txt | head -150
for d in $OUT/p*/; do rm -rf "$d"; done
