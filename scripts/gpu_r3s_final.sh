#!/bin/bash
# Round-3 second-session measurement call: the -m gpu suite + short bench, the PMC passes of the closed step
# (profiles/r3s_pmc_summary.*), and the rocprofv3 kernel stats at the headline, one C5 rank and L = 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
PYTEST_TIMEOUT=700 STEPS=20 bash scripts/gpu_tests.sh || exit $?
PMC_NAME=pmc_r3s bash scripts/pmc_r3.sh > gpurun_out/pmc_r3s.log 2>&1 || { tail -20 gpurun_out/pmc_r3s.log; exit 1; }
tail -5 gpurun_out/pmc_r3s.log
PROF_NAME=${PROF_NAME:-r3s2} CFGS="headline c5rank L2" bash scripts/prof_r3.sh > gpurun_out/prof_r3s2.log 2>&1 || { tail -20 gpurun_out/prof_r3s2.log; exit 1; }
grep -h "ms_per_step\|total kernel" gpurun_out/prof_r3s2.log | cut -c1-200
