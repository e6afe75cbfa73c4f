#!/bin/bash
# Run a selection of GPU tests (TESTS="file::name ..." or a -k expression in K) under per-step time limits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/check
timeout -k 10 ${TLIM:-500} python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} ${K:+-k "$K"} \
  > gpurun_out/check/${NAME:-pytest}.log 2>&1
rc=$?; tail -25 gpurun_out/check/${NAME:-pytest}.log; exit $rc
