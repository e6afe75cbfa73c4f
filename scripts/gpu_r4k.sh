#!/bin/bash
# Round-4: the S GEMM leaving CUs to the ConvVAE stream (LVAE_SYRK_RESERVE) at the headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4k}
mkdir -p $OUT
bench() {  # name env... -- args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 bench.py "$@" --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -20 $OUT/b_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
}
for r in 1 2; do
  for res in 0 8 16 32 64; do
    bench h_r${res}_$r LVAE_SYRK_RESERVE=$res -- --regime closed || exit 1
  done
done
