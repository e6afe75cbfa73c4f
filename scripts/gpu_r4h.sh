#!/bin/bash
# Round-4: the factor's host enqueue on a worker thread (LVAE_ASYNC_FACTOR) -- -m gpu, then share8 / headline A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${PROF_NAME:-r4h}
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
    -p no:cacheprovider --maxfail=5 ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
  [ $rc -le 1 ] || exit $rc
fi
bench() {  # name env... -- args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 bench.py "$@" --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -20 $OUT/b_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
}
for r in 1 2; do
  bench s8_g0_$r LVAE_GRAPH_VAE=0 -- --regime closed --rank-share 8 || exit 1
  bench s8_g1_$r LVAE_GRAPH_VAE=1 -- --regime closed --rank-share 8 || exit 1
  bench s8_g1np_$r LVAE_GRAPH_VAE=1 LVAE_CI_PIPE=0 -- --regime closed --rank-share 8 || exit 1
  bench h_g0_$r LVAE_GRAPH_VAE=0 -- --regime closed || exit 1
  bench h_g1_$r LVAE_GRAPH_VAE=1 -- --regime closed || exit 1
done
NAME=s8_g1 bash scripts/trace_step.sh --rank-share 8 || exit 1
