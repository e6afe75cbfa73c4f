#!/bin/bash
# MFMA utilisation PMC pass over the headline closed bench (one rocprofv3 --pmc run, kernel trace only):
# SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (+ the SQ_INSTS_VALU_MFMA_MOPS_* counters this box lists)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/${NAME:-mfma}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 90 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
C="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for m in SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_BF16; do
  grep -q "$m" $OUT/counters.txt && C="$C $m"
done
grep -q SQ_VALU_MFMA_BUSY_CYCLES $OUT/counters.txt || { echo "no SQ_VALU_MFMA_BUSY_CYCLES on this box"; grep -o "SQ_[A-Z_]*MFMA[A-Z0-9_]*" $OUT/counters.txt | sort -u; exit 1; }
echo "counters: $C"
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/p -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime ${REGIME:-closed} --steps 2 --warmup 1 --h-steps 5 --no-cpu-baseline --no-phase-timing \
  --no-c2 --no-dp-world1 > $OUT/p.json 2> $OUT/p.err || { tail -5 $OUT/p.err; exit 1; }
python3 $ROOT/scripts/mfma_pmc.py $OUT > $OUT/mfma_summary.txt && cat $OUT/mfma_summary.txt
rm -rf $OUT/p
