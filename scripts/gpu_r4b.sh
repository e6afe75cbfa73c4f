#!/bin/bash
# Round-4 A/B call: -m gpu suite, then the rank-share rehearsal (rank 0 of 8: 2 dims, 512 images) and the
# headline under the inverse's schedules: LVAE_CI_PIPE=0 (trtri by recursive doubling after potrf),
# LVAE_CI_PIPE_LAUUM=0 (pipelined trtri), default (pipelined trtri + lauum); optional rocprof of share8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
N=${PROF_NAME:-r4b}
OUT=$ROOT/gpurun_out/$N
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
  env "${envs[@]}" timeout -k 10 300 python3 bench.py "$@" --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -20 $OUT/b_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('phase_ms_per_step',{}).items()})"
}
for r in 1 2; do
  bench share8_p0_$r LVAE_CI_PIPE=0 -- --regime closed --rank-share 8 || exit 1
  bench share8_p1_$r LVAE_CI_PIPE_LAUUM=0 -- --regime closed --rank-share 8 || exit 1
  bench share8_p2_$r X=1 -- --regime closed --rank-share 8 || exit 1
done
bench share4_p0 LVAE_CI_PIPE=0 -- --regime closed --rank-share 4 || exit 1
bench share4_p2 X=1 -- --regime closed --rank-share 4 || exit 1
bench share2_p0 LVAE_CI_PIPE=0 -- --regime closed --rank-share 2 || exit 1
bench share2_p2 LVAE_CI_PIPE_L=8 -- --regime closed --rank-share 2 || exit 1
bench headline X=1 -- --regime closed || exit 1
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  echo "[$(date +%T)] rocprofv3 share8"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof8 -o run --output-format csv -- \
    python3 $ROOT/bench.py --regime closed --rank-share 8 --steps 20 --warmup 5 --no-cpu-baseline --no-c2 \
    > $OUT/prof8.json 2> $OUT/prof8.err || { tail -20 $OUT/prof8.err; exit 1; }
  python3 $ROOT/scripts/kstats.py $OUT/prof8/run_kernel_stats.csv 30 > $OUT/share8_kernel_stats.txt
  cp $OUT/prof8/run_kernel_stats.csv $OUT/share8_kernel_stats.csv
  rm -f $OUT/prof8/run_kernel_trace.csv
  head -16 $OUT/share8_kernel_stats.txt
fi
