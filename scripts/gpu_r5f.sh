#!/bin/bash
# Round 5: the binned route's tests, the KL parity tests that route through it, then the slab pass's part timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r5f; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PYT tests/test_gpu_kl_hyper.py -x -s > $OUT/hyper.log 2>&1; rc=$?
grep -E "passed|failed|rel err|route raw" $OUT/hyper.log | tail -20
[ $rc -eq 0 ] || { grep -E "^E |Error" $OUT/hyper.log | head -30; exit $rc; }
timeout -k 10 400 $PYT tests/test_gpu_regime_b.py -x -k "resid_paths or kernel_variants or vs_oracle or high_cond" > $OUT/kl.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/kl.log | tail -3
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/kl.log | head -30; exit $rc; }
MASKS="${MASKS:-0 1 2 3}" bash $ROOT/scripts/gpu_hbdbg.sh
