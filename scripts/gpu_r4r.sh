#!/bin/bash
# Round 4: the unrolled Gram-adjoint table kernel (kl_gram_bwd_tab2_kernel) -- the Regime B parity tests that
# exercise the adjoint, then the closed bench with LVAE_GRAM_TAB2=0 / 1 alternated, and a rocprof stats pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4r}
mkdir -p $OUT
echo "[$(date +%T)] pytest (Regime B)"
timeout -k 10 500 python -u -m pytest tests/test_gpu_regime_b.py -m gpu -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider --maxfail=3 > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -8
[ $rc -le 1 ] || exit $rc
for r in 1 2; do for v in 0 1; do
  LVAE_GRAM_TAB2=$v timeout -k 10 300 python3 bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/b_${v}_${r}.json 2> $OUT/b_${v}_${r}.err || { tail -20 $OUT/b_${v}_${r}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${v}_${r}.json')); p=d['phase_ms_per_step']; print('TAB2=$v', round(d['ms_per_step'],3), 'gram_bwd', round(p['gram_bwd'],3), 'syrk', round(p['syrk'],3))"
done; done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  LVAE_GRAM_TAB2=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p$v -o run --output-format csv -- \
    python3 $ROOT/bench.py --regime closed --steps 10 --warmup 3 --no-cpu-baseline --no-c2 --no-phase-timing \
    > $OUT/p$v.json 2> $OUT/p$v.err || { tail -20 $OUT/p$v.err; exit 1; }
  grep -h "gram_bwd_tab" $OUT/p$v/run_kernel_stats.csv | cut -c1-160
  rm -f $OUT/p$v/run_kernel_trace.csv
done
