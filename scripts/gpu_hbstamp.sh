#!/bin/bash
# The slab pass's per-section cycle stamps (build_diag/liblvae_hip.so from scripts/build_hbstamp.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/hbstamp; mkdir -p $OUT
for m in ${MASKS:-0}; do
  LVAE_HB_DBG=$m LVAE_LIB=$ROOT/build_diag/liblvae_hip.so timeout -k 10 200 python3 $ROOT/scripts/gram_micro.py 1 > $OUT/stamp_$m.log 2>&1 || exit $?
  echo "== mask $m"; grep "hbstamp J 0 " $OUT/stamp_$m.log | sort -k5 -n | tail -8
done
