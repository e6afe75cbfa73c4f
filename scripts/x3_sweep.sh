#!/bin/bash
# Accuracy / speed of the f16 3-product GEMM engine per kernel class (LVAE_X3 bit mask:
# 1 panel, 2 update, 4 trtri, 8 z, 16 lauum, 32 syrk).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/x3
mkdir -p $OUT
for m in ${MASKS:-0 32 63}; do
  echo "== mask $m"
  LVAE_X3=$m timeout -k 10 300 python -m pytest tests/test_gpu_regime_b.py -q -p no:cacheprovider > $OUT/pytest_$m.log 2>&1
  rc=$?; tail -1 $OUT/pytest_$m.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  LVAE_X3=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$m.json 2> $OUT/bench_$m.err
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/bench_$m.json'));print(d['ms_per_step'], d['phase_ms_per_step'], d['roofline']['achieved'])"
done
