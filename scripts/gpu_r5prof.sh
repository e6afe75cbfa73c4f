#!/bin/bash
# Round 5: the hyper tests on the current build, then the default closed bench command under
# rocprofv3 --kernel-trace --stats (the headline kernel table) and one plain bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r5prof; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PYT tests/test_gpu_kl_hyper.py -x > $OUT/hyper.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/hyper.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |Error" $OUT/hyper.log | head -30; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --no-cpu-baseline --no-c2 --steps 20 --warmup 5 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || exit $?
rm -f $OUT/prof/*kernel_trace.csv
python3 $ROOT/scripts/kstats.py $OUT/prof/run_kernel_stats.csv 30 25
