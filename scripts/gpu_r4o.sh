#!/bin/bash
# Round 4: the bench's clock record (closed bench, un-profiled and under rocprofv3) and one graphed Hensman
# step's kernel timeline (the Regime A critical path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4o}
mkdir -p $OUT
echo "[$(date +%T)] closed bench (clock record)"
timeout -k 10 300 python3 bench.py --regime closed --steps 10 --warmup 3 --no-cpu-baseline --no-c2 \
  > $OUT/b_closed.json 2> $OUT/b_closed.err || { tail -20 $OUT/b_closed.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_closed.json')); print(round(d['ms_per_step'],3), d.get('clock'), d['roofline']['avg_launch_us_event'])"
cd /tmp && export TMPDIR=/tmp
echo "[$(date +%T)] the same under rocprofv3 --kernel-trace --stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/pc -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --steps 10 --warmup 3 --no-cpu-baseline --no-c2 \
  > $OUT/b_closed_prof.json 2> $OUT/b_closed_prof.err || { tail -20 $OUT/b_closed_prof.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_closed_prof.json')); print(round(d['ms_per_step'],3), d.get('clock'), d['roofline']['avg_launch_us_event'])"
grep syrk_c16 $OUT/pc/run_kernel_stats.csv | cut -c1-200
rm -f $OUT/pc/run_kernel_trace.csv
echo "[$(date +%T)] graphed Hensman step trace"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/h -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime hensman --steps 1 --warmup 1 --h-steps 30 --no-cpu-baseline --no-phase-timing \
  --no-c2 > $OUT/h.json 2> $OUT/h.err || { tail -5 $OUT/h.err; exit 1; }
python3 $ROOT/scripts/timeline.py $OUT/h/run_kernel_trace.csv hn_reduce > $OUT/hensman_timeline.txt
python3 $ROOT/scripts/hensman_trace.py $OUT/h/run_kernel_trace.csv > $OUT/hensman_steps.txt
rm -f $OUT/h/run_kernel_trace.csv
head -3 $OUT/hensman_timeline.txt; head -12 $OUT/hensman_steps.txt
