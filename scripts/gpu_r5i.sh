#!/bin/bash
# Round 5: the glue / ConvVAE tests, then one step's kernel timeline (scripts/gpu_timeline.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r5i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_glue.py tests/test_gpu_regime_b.py -k "glue or fused or closed_step or vae" -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" $OUT/pytest.log | tail -6
[ $rc -eq 0 ] || { grep -E "^E " $OUT/pytest.log | head -20; exit $rc; }
bash $ROOT/scripts/gpu_timeline.sh
