#!/bin/bash
# Round 5: the whole -m gpu suite, then the default closed bench (warms MIOpen's perf db for this box),
# then the same bench command under rocprofv3 --kernel-trace --stats (the headline kernel table).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/${NAME:-r5g}; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    --maxfail=5 ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 400 python3 bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', round(d['ms_per_step'],3), 'ms', d.get('hyper_route'), {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
rm -f $OUT/prof/*kernel_trace.csv
cp $OUT/prof/run_kernel_stats.csv $OUT/headline_kernel_stats.csv
python3 $ROOT/scripts/kstats.py $OUT/prof/run_kernel_stats.csv 40 25 > $OUT/headline_kernel_stats.txt
head -32 $OUT/headline_kernel_stats.txt
