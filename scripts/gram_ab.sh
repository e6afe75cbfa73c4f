#!/bin/bash
# A/B kernel stats of the exact-KL forward + backward alone (scripts/gram_micro.py):
# build_ab/liblvae_hip.so vs the tree's library (swapped in the box's scratch copy).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; SO=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so
cp $SO /tmp/new.so
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  if [ $v = old ]; then cp $ROOT/build_ab/liblvae_hip.so $SO; else cp /tmp/new.so $SO; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ab_$v -o run --output-format csv -- \
    python3 $ROOT/scripts/gram_micro.py 5 || exit $?
  rm -f $OUT/ab_$v/*kernel_trace.csv
done
cp /tmp/new.so $SO
