#!/bin/bash
# Round 4: the early decoder backward -- the closed-step tests, then LVAE_EARLY_DEC=0 / 1 alternated (3 rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4v}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -m gpu -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "orders_agree or graphed_closed or closed_step" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR|Error" $OUT/pytest.log | tail -8
[ $rc -le 1 ] || exit $rc
for r in 1 2 3; do for v in 0 1; do
  LVAE_EARLY_DEC=$v timeout -k 10 300 python3 bench.py --regime closed --steps 20 --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/b_${v}_${r}.json 2> $OUT/b_${v}_${r}.err || { tail -20 $OUT/b_${v}_${r}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${v}_${r}.json')); p=d['phase_ms_per_step']; print('early_dec=$v', round(d['ms_per_step'],3), 'syrk', round(p['syrk'],3), 'gram_bwd', round(p['gram_bwd'],3), d.get('clock',{}).get('gfx_mhz_median'))"
done; done
