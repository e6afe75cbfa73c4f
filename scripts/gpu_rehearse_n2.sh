#!/bin/bash
# The default N = 2 bench line rehearsed on the one-GPU box: two ranks on cuda:0 over gloo (timings meaningless)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/n2
LVAE_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --h-steps 20 \
  > gpurun_out/n2/bench.json 2> gpurun_out/n2/bench.err || { tail -30 gpurun_out/n2/bench.err; exit 1; }
python3 -c "
import json; d = json.load(open('gpurun_out/n2/bench.json'))
print('closed', d['n_gpus'], round(d['ms_per_step'], 3), 'ms', d['config'].get('parallelism'))
ra = d.get('regime_a', {}); print('regime_a', {k: ra.get(k) for k in ('value', 'ms_per_step', 'samples_per_sec', 'scaling', 'error')})"
