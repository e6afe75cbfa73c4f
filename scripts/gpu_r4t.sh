#!/bin/bash
# Round 4: the cheap refinement gate -- the -m gpu suite, then the closed bench with LVAE_SYRK_RESERVE 0 / 32
# alternated (3 rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4t}
mkdir -p $OUT
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider --maxfail=5 > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -8
[ $rc -le 1 ] || exit $rc
for r in 1 2 3; do for v in 0 32; do
  LVAE_SYRK_RESERVE=$v timeout -k 10 300 python3 bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/b_${v}_${r}.json 2> $OUT/b_${v}_${r}.err || { tail -20 $OUT/b_${v}_${r}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${v}_${r}.json')); p=d['phase_ms_per_step']; print('reserve=$v', round(d['ms_per_step'],3), 'syrk', round(p['syrk'],3), 'gram_bwd', round(p['gram_bwd'],3), 'reduce', round(p['kl_reduce'],3), d.get('clock',{}).get('gfx_mhz_median'))"
done; done
