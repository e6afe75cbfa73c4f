#!/bin/bash
# Same-box A/B of the graphed Hensman step: the tree's library (new) vs build_ab (old), alternated x3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r4ab; mkdir -p $OUT
SO=$ROOT/longitudinal-vae_amd/lvae_amd/liblvae_hip.so
cp $SO /tmp/new.so
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then cp $ROOT/build_ab/liblvae_hip.so $SO; else cp /tmp/new.so $SO; fi
    timeout -k 10 300 python3 bench.py --regime hensman --steps 1 --warmup 1 --h-steps 100 --no-cpu-baseline --no-c2 \
      > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail -20 $OUT/b_${v}_$r.err; cp /tmp/new.so $SO; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$r.json')); print('$v', d.get('ms_per_step'))"
  done
done
cp /tmp/new.so $SO
