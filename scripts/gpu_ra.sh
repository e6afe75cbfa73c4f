#!/bin/bash
# Regime A checks: the RCCL / two-graph tests, the Regime A suite, then the bench's Regime A line with its
# data-parallel world-1 RCCL sub-record
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ra
TESTS="tests/test_gpu_rccl.py tests/test_gpu_regime_a.py" NAME=ra_tests TLIM=600 bash scripts/gpu_check.sh || exit 1
timeout -k 10 300 python3 bench.py --regime hensman --no-cpu-baseline --dp-world1 > gpurun_out/ra/ra.json 2> gpurun_out/ra/ra.err || { tail -20 gpurun_out/ra/ra.err; exit 1; }
python3 -c "
import json; d = json.load(open('gpurun_out/ra/ra.json'))
print('regime A', round(d['ms_per_step'], 3), 'ms; dp world-1 RCCL', d.get('dp_world1_rccl'))"
