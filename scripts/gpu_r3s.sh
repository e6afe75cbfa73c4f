#!/bin/bash
# Round-3 second-session GPU call: the -m gpu suite + a short bench (scripts/gpu_tests.sh), then the
# potrf pivots' phase timestamps (scripts/pivot_prof.py) at L = 16 and L = 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  bash scripts/gpu_tests.sh || exit $?
fi
echo "[$(date +%T)] pivot phases"
timeout -k 10 180 python -u scripts/pivot_prof.py > $OUT/pivot_prof.txt 2>&1
rc=$?; cat $OUT/pivot_prof.txt; exit $rc
