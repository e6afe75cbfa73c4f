#!/bin/bash
# Per-rank evidence for the latent-sharded step: rocprofv3 kernel stats of the closed step at L = 2
# (one 8-GPU rank's latent dims, all N images on the one GPU), and a 4-rank gloo rehearsal of the
# sharded step on the one GPU (correctness of the 4-rank path; ranks share the GPU, so no timing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# one unprofiled run first: a fresh box has no MIOpen find-db, and MIOpen's Find (hundreds of
# candidate-solver kernels, fp64 naive reference convs among them) would otherwise land in the profile
timeout -k 10 300 python bench.py --regime closed --L 2 --steps 2 --warmup 1 --no-cpu-baseline --no-c2 > /dev/null 2>&1 || exit $?
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/r2s_L2_prof -o run \
  --output-format csv -- python3 $ROOT/bench.py --regime closed --L 2 --steps 5 --warmup 2 --no-cpu-baseline \
  --no-phase-timing --no-c2 > $OUT/r2s_L2_prof_bench.json 2> $OUT/r2s_L2_prof.err ) || exit $?
rm -f $OUT/r2s_L2_prof/*kernel_trace.csv
[ "${W4:-1}" = "1" ] || exit 0
LVAE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 3 --warmup 1 --h-steps 10 \
  > $OUT/r2s_w4.json 2> $OUT/r2s_w4.err || { tail -20 $OUT/r2s_w4.err; exit 1; }
cat $OUT/r2s_w4.json | head -c 600; echo
grep -E "rank [0-9]: dims" $OUT/r2s_w4.err | cut -c1-120
