#!/bin/bash
# Gram adjoint chunk tables: same-box A/B of the kernel stats (old = build_ab, new = tree), the
# hyper-gradients of both printed for the bit-identity check, then the Regime B GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r4x; mkdir -p $OUT
SO=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so
cp $SO /tmp/new.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $ROOT/scripts/gram_micro.py 2 > $OUT/warm.log 2>&1 || exit $?
for v in old new old new; do
  if [ $v = old ]; then cp $ROOT/build_ab/liblvae_hip.so $SO; else cp /tmp/new.so $SO; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ab_$v -o run --output-format csv -- \
    python3 $ROOT/scripts/gram_micro.py 5 > $OUT/micro_$v.log 2>&1 || exit $?
  grep -h "kl_gram_bwd_tab\|gram_sq_fill_tab" $OUT/ab_$v/*/run_kernel_stats.csv $OUT/ab_$v/run_kernel_stats.csv 2>/dev/null | cut -c1-200 >> $OUT/stats_$v.txt
  rm -f $OUT/ab_$v/*kernel_trace.csv $OUT/ab_$v/*/*kernel_trace.csv
done
cp /tmp/new.so $SO
cd $ROOT && timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_regime_b.py > $OUT/pytest_b.log 2>&1
echo "pytest rc $?" >> $OUT/pytest_b.log
tail -3 $OUT/pytest_b.log
grep -h "hyper-grads" $OUT/micro_*.log
