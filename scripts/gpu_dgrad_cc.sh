#!/bin/bash
# Dev A/B: conv3x3_pool_dgrad_kernel's LDS stage (LVAE_DGRAD_CC channels; 0 = all) -- parity tests, the op alone.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/dgradcc; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_regime_b.py \
  -x -k "dgrad or conv_relu_maxpool2" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head; exit $rc; }
for cc in 16 0 8 16 0 8; do
  echo -n "CC=$cc "; LVAE_DGRAD_CC=$cc timeout -k 10 120 python3 scripts/dgrad_ab.py 2>&1 | grep -v amdgpu.ids | grep -E "^hip" | tr '\n' ' '; echo
done
