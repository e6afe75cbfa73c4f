#!/bin/bash
# Regime A with the Hensman prior launched beside the ConvVAE forward: the Regime A GPU tests, then
# the graphed step's time (3 runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r4z; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_regime_a.py > $OUT/pytest_a.log 2>&1; rc=$?
tail -3 $OUT/pytest_a.log
[ $rc -eq 0 ] || exit $rc
SO=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --regime hensman --steps 1 --warmup 1 --h-steps 100 --no-cpu-baseline --no-c2 \
    > $OUT/b_hens_$r.json 2> $OUT/b_hens_$r.err || { tail -20 $OUT/b_hens_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_hens_$r.json')); print('hensman', d.get('ms_per_step'))"
done
