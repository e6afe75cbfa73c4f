#!/bin/bash
# A/B of the closed step at several per-GPU latent-dim counts: build_ab/liblvae_hip.so (previous sweep
# schedule) vs the tree's library.  Swaps the library file in the box's scratch copy.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out; mkdir -p $OUT; SO=longitudinal-vae_amd/lvae_amd/liblvae_hip.so
cp $SO /tmp/new.so
for v in ${VARIANTS:-old new}; do
  if [ $v = old ]; then cp build_ab/liblvae_hip.so $SO; else cp /tmp/new.so $SO; fi
  for L in ${LS:-2 4 16}; do
    timeout -k 10 200 python bench.py --regime closed --L $L --steps 10 --warmup 3 --no-cpu-baseline --no-c2 \
      > $OUT/ab_${v}_L$L.json 2> $OUT/ab_${v}_L$L.err || exit $?
    python -c "import json,sys; d=json.load(open('$OUT/ab_${v}_L$L.json')); print('$v', 'L=$L', round(d['ms_per_step'],3), {k: round(x,3) for k, x in d['phase_ms_per_step'].items()})"
  done
done
cp /tmp/new.so $SO
