#!/bin/bash
# r2s GPU pass: full -m gpu suite, default bench (+ rocprof of the closed step), an L = 2 closed-step
# bench (the per-rank load of the 8-GPU latent-sharded step), and the 2-rank gloo rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out; mkdir -p $OUT; TAG=${TAG:-r2s}
stage() { echo "[$(date +%T)] $*"; }
if [ "${TESTS:-1}" = "1" ]; then
  stage pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${K:+-k "$K"} > $OUT/${TAG}_pytest.log 2>&1
  rc=$?; stage "pytest rc=$rc"; tail -4 $OUT/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SMALL_L:-1}" = "1" ]; then
  stage "bench L=2"
  timeout -k 10 300 python bench.py --regime closed --L 2 --steps 10 --warmup 3 --no-cpu-baseline --no-c2 \
    > $OUT/${TAG}_bench_L2.json 2> $OUT/${TAG}_bench_L2.err
  rc=$?; stage "bench L=2 rc=$rc"; cat $OUT/${TAG}_bench_L2.json | head -c 1500; echo; [ $rc -eq 0 ] || exit $rc
fi
TAG=$TAG REHEARSE=${REHEARSE:-1} BENCH=${BENCH:-1} PROF=${PROF:-1} bash scripts/gpu_session.sh
