#!/bin/bash
# One round's GPU evidence, in order (TAG names the files, e.g. r6): the -m gpu suite, smoke, the headline kernel
# profile (rocprofv3 --kernel-trace --stats of the closed bench after an un-profiled warm-up run: MIOpen's find
# outside the window; .csv and .txt from that ONE run), FETCH / WRITE PMC passes, the MFMA-busy pass, the binned
# slab pass's SQ counters, then the default bench line priced on THIS run's profile files (copied to profiles/).
# SKIP_TESTS=1: the suite and smoke are skipped.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${TAG:-r6}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/ev_$TAG; mkdir -p $OUT
PYT="python -u -m pytest -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 1000 $PYT tests -m gpu > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
  [ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest_gpu.log | head -20; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 400 python3 bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/warm.json 2> $OUT/warm.err || { tail -20 $OUT/warm.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
cp $OUT/prof/run_kernel_stats.csv $OUT/headline_kernel_stats.csv
python3 $ROOT/scripts/kstats.py $OUT/prof/run_kernel_stats.csv 40 25 > $OUT/headline_kernel_stats.txt
rm -f $OUT/prof/*kernel_trace.csv
head -8 $OUT/headline_kernel_stats.txt
cd $ROOT
PMC_NAME=ev_$TAG/pmc bash scripts/pmc.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
NAME=ev_$TAG/mfma bash scripts/gpu_mfma_pmc.sh > $OUT/mfma.log 2>&1 || { tail -20 $OUT/mfma.log; exit 1; }
MASKS=0 bash scripts/gpu_hbpmc.sh > $OUT/hbpmc.txt 2>&1 || { tail -20 $OUT/hbpmc.txt; exit 1; }
# the bench line reads profiles/${TAG}_*: this run's files (the same ones get committed)
cp $OUT/headline_kernel_stats.csv profiles/${TAG}_headline_kernel_stats.csv
cp $OUT/headline_kernel_stats.txt profiles/${TAG}_headline_kernel_stats.txt
cp $OUT/pmc/pmc_summary.json profiles/${TAG}_pmc_summary.json
cp $OUT/pmc/pmc_summary.txt profiles/${TAG}_pmc_summary.txt
cp $OUT/mfma/mfma_summary.json profiles/${TAG}_mfma_pmc.json
cp $OUT/mfma/mfma_summary.txt profiles/${TAG}_mfma_pmc.txt
timeout -k 10 900 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/bench_default.json'))
print('default bench', round(d['ms_per_step'], 3), 'ms', d['roofline']['kernel'][:40], 'frac', round(d['roofline']['frac'], 3))
ra = d.get('regime_a') or {}
print('cpu', d.get('cpu_baseline', {}).get('value'), 'regime_a', ra.get('ms_per_step'), 'dp1', (ra.get('dp_world1_rccl') or {}).get('ms_per_step'))
print('c2', {k: d.get('c2', {}).get('potrf_export', {}).get(k) for k in ('speedup_f32', 'speedup_f64', 'lvae_potrf_f64_ms', 'torch_cholesky_f64_ms')})"
