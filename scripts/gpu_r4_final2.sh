#!/bin/bash
# Round-4 headline profile, redone with MIOpen's find database warm (gpu_r4_final.sh profiled the first
# run on a fresh box: MIOpen's Find benchmarks polluted the per-step totals):
#   1. one closed bench run (warms MIOpen's find DB, not kept)
#   2. rocprofv3 --kernel-trace --stats of the closed bench at the default command's steps / warm-up
#      (10 / 3), no CPU leg, no C2 -> profiles/r4_headline_kernel_stats.{csv,txt}
#   3. the default bench line (CPU baseline, C2 and Regime A included), which reads that summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4f2}
mkdir -p $OUT
echo "[$(date +%T)] warm-up run"
timeout -k 10 300 python3 bench.py --regime closed --steps 10 --warmup 3 --no-cpu-baseline --no-c2 \
  > $OUT/warm.json 2> $OUT/warm.err || { tail -20 $OUT/warm.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
echo "[$(date +%T)] rocprofv3 kernel trace of the closed bench"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --steps 10 --warmup 3 --no-cpu-baseline --no-c2 \
  > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
cp $OUT/prof/run_kernel_stats.csv $OUT/headline_kernel_stats.csv
python3 $ROOT/scripts/kstats.py $OUT/headline_kernel_stats.csv 30 > $OUT/headline_kernel_stats.txt
cp $OUT/headline_kernel_stats.csv $ROOT/profiles/r4_headline_kernel_stats.csv
rm -f $OUT/prof/run_kernel_trace.csv
head -12 $OUT/headline_kernel_stats.txt
python3 -c "import json; d=json.load(open('$OUT/prof.json')); print('profiled run', round(d['ms_per_step'],3), 'ms; S GEMM event avg', d['roofline'].get('avg_launch_us_event'))"
cd $ROOT
echo "[$(date +%T)] default bench"
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], 'frac', r['frac'], 'frac_event', r['frac_event'], r['avg_launch_us'], r['avg_launch_us_event'])"
