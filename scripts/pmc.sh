#!/bin/bash
# rocprofv3 PMC passes over the Regime B bench step (kernel trace only, one counter group per run:
# MI355X_MICROARCH.md -- FETCH_SIZE and WRITE_SIZE never share a pass).  Summary -> $OUT/pmc_summary.*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PMC_NAME:-pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ "${LIST:-0}" = "1" ]; then
  timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
fi
PASSES=${PASSES:-"FETCH_SIZE;WRITE_SIZE"}
IFS=';' read -ra P <<< "$PASSES"
i=0
for c in "${P[@]}"; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $c"
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $OUT/p$i -o run --output-format csv -- \
    python3 $ROOT/bench.py --regime ${PMC_REGIME:-closed} --steps 2 --warmup 1 --h-steps 5 --no-cpu-baseline \
    --no-phase-timing --no-c2 > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; exit 1; }
done
python3 $ROOT/scripts/pmc_summary.py $OUT > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt | head -150
for d in $OUT/p*/; do rm -rf "$d"; done
