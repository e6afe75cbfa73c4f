#!/bin/bash
# Dev A/B of the pivot's panel variant: per-panel stamps (build_pv: -DLVAE_PV_STAMP_CHOL), the inverse's time with
# the tree's library vs build_p0 (-DLVAE_PV_PANEL2B=0), then the inverse / KL parity tests on the tree's library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/panel_ab; mkdir -p $OUT
LVAE_LIB=$ROOT/build_pv/liblvae_hip.so timeout -k 10 200 python3 scripts/pivot_prof_chol.py 2>&1 | grep -v amdgpu.ids || exit 1
for L in 2 16; do
  for lib in tree p0 tree p0; do
    if [ $lib = tree ]; then LIBP=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so; else LIBP=$ROOT/build_$lib/liblvae_hip.so; fi
    echo -n "$lib: "; L=$L LVAE_LIB=$LIBP timeout -k 10 120 python3 scripts/inv_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_regime_b.py \
  -x -k "spd_inverse or vs_oracle or high_cond or small_noise" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -2; exit $rc
