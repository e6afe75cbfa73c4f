#!/bin/bash
# Round-4 final measurement call: the whole -m gpu suite, then gpu_r4_final2.sh (warm-up run, rocprofv3 kernel
# stats of the closed bench at the default steps -> profiles/r4_headline_kernel_stats.*, the default bench line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4f3}
mkdir -p $OUT
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -8
[ $rc -le 1 ] || exit $rc
PROF_NAME=${PROF_NAME:-r4f3} bash scripts/gpu_r4_final2.sh
