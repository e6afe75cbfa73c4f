#!/bin/bash
# Dev A/B: lauum / trtri-X chunks from the end of their K ranges (the tree) vs in order (build_kf: -DLVAE_CI_KREV=0):
# parity tests on the tree's library, the inverse alone, kernel stats, and interleaved closed-bench rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/krev; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_regime_b.py \
  tests/test_gpu_kl_hyper.py -x -k "spd_inverse or vs_oracle or high_cond or small_noise or deterministic or routes" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head; exit $rc; }
for L in 16 2; do
  for lib in tree kf tree kf; do
    if [ $lib = tree ]; then LIBP=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so; else LIBP=$ROOT/build_$lib/liblvae_hip.so; fi
    echo -n "$lib: "; L=$L LVAE_LIB=$LIBP timeout -k 10 120 python3 scripts/inv_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in tree kf; do
  if [ $lib = tree ]; then LIBP=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so; else LIBP=$ROOT/build_$lib/liblvae_hip.so; fi
  L=16 REPS=5 LVAE_LIB=$LIBP timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$lib -o run --output-format csv -- \
    python3 $ROOT/scripts/inv_ab.py > $OUT/p$lib.log 2>&1 || exit 1
  rm -f $OUT/p$lib/*kernel_trace.csv
  echo "== $lib"; python3 $ROOT/scripts/kstats.py $OUT/p$lib/run_kernel_stats.csv 12 8 | grep -E "gemm_kernel"
done
