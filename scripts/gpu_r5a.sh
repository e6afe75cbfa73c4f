#!/bin/bash
# Round 5, first box: the new N x N factor / solve tests and the changed tests first, then the whole -m gpu
# suite, then a default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r5a; mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PYT tests/test_gpu_linalg.py -x -s > $OUT/linalg.log 2>&1; rc=$?
grep -E "passed|failed|error" $OUT/linalg.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 $PYT tests -m gpu -s > $OUT/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
grep -E "hensman kernel variants rel" $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d.get('c2',{}).get('potrf_export')), json.dumps(d.get('cpu_baseline',{}).get('sample')))"
