#!/bin/bash
# Round-4: C5 at one rank's share (rank 0 of 8: N = 16384, L = 32 / 8 = 4 dims, 2048 images) -- bench line and
# rocprofv3 kernel stats over the timed steps (MIOpen's find done in the warm-up), plus share8 / headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4j}
mkdir -p $OUT
echo "[$(date +%T)] C5 rank share bench"
timeout -k 10 400 python3 bench.py --regime closed --P 1024 --L 32 --rank-share 8 --steps 10 --warmup 3 --no-cpu-baseline --no-c2 \
  > $OUT/c5share.json 2> $OUT/c5share.err || { tail -20 $OUT/c5share.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c5share.json').read().strip().splitlines()[-1]); print('c5share', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
cd /tmp && export TMPDIR=/tmp
echo "[$(date +%T)] rocprofv3 C5 rank share"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/c5prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --P 1024 --L 32 --rank-share 8 --steps 10 --warmup 3 --no-cpu-baseline --no-c2 \
  > $OUT/c5prof.json 2> $OUT/c5prof.err || { tail -20 $OUT/c5prof.err; exit 1; }
python3 $ROOT/scripts/kstats.py $OUT/c5prof/run_kernel_stats.csv 30 > $OUT/c5share_kernel_stats.txt
cp $OUT/c5prof/run_kernel_stats.csv $OUT/c5share_kernel_stats.csv
python3 $ROOT/scripts/timeline.py $OUT/c5prof/run_kernel_trace.csv > $OUT/c5share_timeline.txt
rm -f $OUT/c5prof/run_kernel_trace.csv
head -14 $OUT/c5share_kernel_stats.txt; head -2 $OUT/c5share_timeline.txt
python3 -c "import json; d=json.loads(open('$OUT/c5prof.json').read().strip().splitlines()[-1]); print('c5share (profiled)', round(d['ms_per_step'],3), 'ms')"
