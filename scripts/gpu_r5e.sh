#!/bin/bash
# Round 5: the binned route's tests, then the slab pass's part timings (scripts/gpu_hbdbg.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r5e; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PYT tests/test_gpu_kl_hyper.py -x -s > $OUT/hyper.log 2>&1; rc=$?
grep -E "passed|failed|rel err|route raw" $OUT/hyper.log | tail -20
[ $rc -eq 0 ] || { grep -E "^E |Error" $OUT/hyper.log | head -30; exit $rc; }
MASKS="${MASKS:-0 1 2 3}" bash $ROOT/scripts/gpu_hbdbg.sh
