#!/bin/bash
# Round-3 third-session measurement call: the whole -m gpu suite, the PMC passes of the closed step
# (profiles/r3s3_pmc_summary.*), the rocprofv3 kernel stats at the headline, one C5 rank and L = 2, and the
# default bench line (CPU baseline included).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
PYTEST_TIMEOUT=700 SKIP_BENCH=1 bash scripts/gpu_tests.sh || exit $?
PMC_NAME=pmc_${PROF_NAME:-r3s3} bash scripts/pmc_r3.sh > gpurun_out/pmc_${PROF_NAME:-r3s3}.log 2>&1 || { tail -20 gpurun_out/pmc_${PROF_NAME:-r3s3}.log; exit 1; }
tail -3 gpurun_out/pmc_${PROF_NAME:-r3s3}.log
PROF_NAME=${PROF_NAME:-r3s3} CFGS="headline c5rank L2" bash scripts/prof_r3.sh > gpurun_out/prof_${PROF_NAME:-r3s3}.log 2>&1 || { tail -20 gpurun_out/prof_${PROF_NAME:-r3s3}.log; exit 1; }
grep -h "ms_per_step\|total kernel" gpurun_out/prof_${PROF_NAME:-r3s3}.log | cut -c1-200
echo "[$(date +%T)] default bench"
timeout -k 10 600 python3 bench.py > gpurun_out/${PROF_NAME:-r3s3}_bench.json 2> gpurun_out/${PROF_NAME:-r3s3}_bench.err || { tail -20 gpurun_out/${PROF_NAME:-r3s3}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${PROF_NAME:-r3s3}_bench.json
