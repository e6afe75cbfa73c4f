#!/bin/bash
# Dev A/B: conv2's weight gradient on a side stream beside its input gradient (the tree) vs one after the other
# (LVAE_CONV_BWD_FORK=0): the conv tests, then interleaved closed-regime bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/fork; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_regime_b.py tests/test_gpu_glue.py \
  -x -k "dgrad or conv_relu_maxpool2 or closed_step or graph or vae" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head; exit $rc; }
for r in 1 2 3; do
  for f in 1 0; do
    LVAE_CONV_BWD_FORK=$f timeout -k 10 240 python3 bench.py --regime closed --steps 30 --warmup 5 --no-cpu-baseline --no-c2 > $OUT/b${f}_$r.json 2> $OUT/b${f}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('fork=$f', d['ms_per_step'])" $OUT/b${f}_$r.json
  done
done
