#!/bin/bash
# Regime A (Hensman step, one HIP graph per step): rocprofv3 --kernel-trace --stats of the bench's Regime A line after
# an un-profiled warm-up run -> gpurun_out/hprof/hensman_kernel_stats.{csv,txt}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/hprof; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --regime hensman --no-cpu-baseline --no-dp-world1 > $OUT/warm.json 2> $OUT/warm.err || { tail -5 $OUT/warm.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime hensman --no-cpu-baseline --no-dp-world1 --h-steps 100 > $OUT/prof.json 2> $OUT/prof.err || { tail -5 $OUT/prof.err; exit 1; }
cp $OUT/prof/run_kernel_stats.csv $OUT/hensman_kernel_stats.csv
python3 $ROOT/scripts/kstats.py $OUT/prof/run_kernel_stats.csv 40 ${KSTEPS:-105} > $OUT/hensman_kernel_stats.txt
python3 $ROOT/scripts/timeline.py $OUT/prof/run_kernel_trace.csv ${MARK:-gram_multi} > $OUT/hensman_timeline.txt 2>&1 || true
rm -f $OUT/prof/*kernel_trace.csv
head -30 $OUT/hensman_kernel_stats.txt
