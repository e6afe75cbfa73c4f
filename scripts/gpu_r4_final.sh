#!/bin/bash
# Round-4 measurement call on the final tree:
#   1. the whole -m gpu suite
#   2. rocprofv3 --kernel-trace --stats of the closed bench (the default command's regime, steps and
#      warm-up; no CPU leg, no C2) -> profiles/r4_headline_kernel_stats.{csv,txt}, which bench.py's
#      roofline reads (frac from the committed profile, frac_event from its own HIP events)
#   3. FETCH_SIZE / WRITE_SIZE passes of the closed step -> profiles/r4_pmc_summary.{json,txt}
#   4. the default bench line (CPU baseline and C2 included), reading the two summaries above
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
N=${PROF_NAME:-r4f}
OUT=$ROOT/gpurun_out/$N
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
  [ $rc -le 1 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp
echo "[$(date +%T)] rocprofv3 kernel trace of the closed bench"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 \
  > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
cp $OUT/prof/run_kernel_stats.csv $OUT/headline_kernel_stats.csv
python3 $ROOT/scripts/kstats.py $OUT/headline_kernel_stats.csv 30 > $OUT/headline_kernel_stats.txt
cp $OUT/headline_kernel_stats.csv $ROOT/profiles/r4_headline_kernel_stats.csv
rm -f $OUT/prof/run_kernel_trace.csv
head -8 $OUT/headline_kernel_stats.txt
cd $ROOT
echo "[$(date +%T)] PMC passes"
PMC_NAME=$N/pmc PASSES="FETCH_SIZE;WRITE_SIZE" bash scripts/pmc_r3.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
cp $OUT/pmc/pmc_summary.json $ROOT/profiles/r4_pmc_summary.json
cp $OUT/pmc/pmc_summary.txt $ROOT/profiles/r4_pmc_summary.txt
grep -i "syrk" $OUT/pmc/pmc_summary.txt | head -4
echo "[$(date +%T)] default bench"
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:700]); print(json.dumps(d.get('c2'))[:500])"
echo "[$(date +%T)] closed bench with every dim's diag(K^-1) refined (LVAE_KL_REFINE=1: the cost of the fp64 path)"
LVAE_KL_REFINE=1 timeout -k 10 300 python3 bench.py --regime closed --steps 5 --warmup 2 --no-cpu-baseline --no-c2 \
  > $OUT/b_refine_all.json 2> $OUT/b_refine_all.err || { tail -20 $OUT/b_refine_all.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_refine_all.json')); print('refine-all', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
