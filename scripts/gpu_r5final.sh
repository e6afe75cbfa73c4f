#!/bin/bash
# Round 5 final evidence, in order: the -m gpu suite, smoke, the headline kernel profile (rocprofv3 --stats of the
# closed bench after a warm-up run: MIOpen's find outside the window), FETCH / WRITE PMC passes, the binned slab
# pass's SQ counters, then the default bench line (CPU leg, C2, Regime A) priced on THIS run's profile files.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/${NAME:-r5final}; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 $PYT tests -m gpu > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" $OUT/pytest_gpu.log | tail -3
  [ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest_gpu.log | head -20; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 400 python3 bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/warm.json 2> $OUT/warm.err || { tail -20 $OUT/warm.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
rm -f $OUT/prof/*kernel_trace.csv
cp $OUT/prof/run_kernel_stats.csv $OUT/headline_kernel_stats.csv
python3 $ROOT/scripts/kstats.py $OUT/prof/run_kernel_stats.csv 40 25 > $OUT/headline_kernel_stats.txt
head -12 $OUT/headline_kernel_stats.txt
cd $ROOT
PMC_NAME=${NAME:-r5final}/pmc bash scripts/pmc.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
MASKS=0 bash scripts/gpu_hbpmc.sh > $OUT/hbpmc.txt 2>&1 || { tail -20 $OUT/hbpmc.txt; exit 1; }
cat $OUT/hbpmc.txt
# the bench line reads profiles/r5_*: this run's files (the same ones get committed)
cp $OUT/headline_kernel_stats.csv profiles/r5_headline_kernel_stats.csv
cp $OUT/pmc/pmc_summary.json profiles/r5_pmc_summary.json
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/bench_default.json'))
print('default bench', round(d['ms_per_step'], 3), 'ms', d['roofline']['kernel'][:40], 'frac', round(d['roofline']['frac'], 3))
print('cpu', d.get('cpu_baseline', {}).get('value'), 'regime_a', (d.get('regime_a') or {}).get('ms_per_step'))"
