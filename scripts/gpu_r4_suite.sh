#!/bin/bash
# The whole -m gpu suite and smoke() on the final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r4suite; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
