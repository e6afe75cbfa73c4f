#!/bin/bash
# Dev A/B: images per block of the encoder convs' weight-gradient kernel (LVAE_WGRAD_PER = 4, the default at
# N >= 2048; 2; 1): parity tests with each, then interleaved closed-regime bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/wgradper; mkdir -p $OUT
for v in 4 2 1; do
  LVAE_WGRAD_PER=$v timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_regime_b.py -x -k "dgrad or conv_relu_maxpool2" > $OUT/tests$v.log 2>&1; rc=$?
  grep -E "passed|failed" $OUT/tests$v.log | tail -1; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests$v.log | head; exit $rc; }
done
for r in 1 2 3; do
  for v in 4 2 1; do
    LVAE_WGRAD_PER=$v timeout -k 10 240 python3 bench.py --regime closed --steps 30 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/b${v}_$r.json 2> $OUT/b${v}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('per=$v', d['ms_per_step'])" $OUT/b${v}_$r.json
  done
done
