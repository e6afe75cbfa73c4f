#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE passes of the closed step at one C5 rank's share (--P 1024 --L 4), counters
# collected for the KL kernels only (--kernel-include-regex: the 16384-image ConvVAE's ~10^5 MIOpen
# dispatches per step are left out), with a ticker so the long MIOpen warm-up shows progress.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_c5; mkdir -p $OUT
( while sleep 45; do date +%T >> $ROOT/gpurun_out/pmc_c5_tick.log; done ) & TICK=$!
trap "kill $TICK 2>/dev/null" EXIT
timeout -k 10 400 python3 $ROOT/bench.py --regime closed --P 1024 --L 4 --steps 1 --warmup 1 --no-cpu-baseline \
  --no-phase-timing --no-c2 > $OUT/warm.json 2> $OUT/warm.err || { tail -5 $OUT/warm.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $c"
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex "syrk|ci_|kl_|gram_|rb_" \
    -d $OUT/p$i -o run --output-format csv -- python3 $ROOT/bench.py --regime closed --P 1024 --L 4 --steps 2 \
    --warmup 1 --no-cpu-baseline --no-phase-timing --no-c2 > $OUT/p$i.json 2> $OUT/p$i.err \
    || { echo "pass $i failed"; tail -5 $OUT/p$i.err; exit 1; }
done
PMC_STEPS=3 PMC_KERNELS="syrk,ci_,kl_,gram_" python3 $ROOT/scripts/pmc_summary.py $OUT > $OUT/pmc_summary.txt
head -40 $OUT/pmc_summary.txt
for d in $OUT/p*/; do rm -rf "$d"; done
