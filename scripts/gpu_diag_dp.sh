#!/bin/bash
# scripts/dp_replay_diag.py variants (the data-parallel two-graph Hensman replay), each in its own process
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/diag
run() { # name env...
  local n=$1; shift
  env "$@" timeout -k 10 150 python3 -u scripts/dp_replay_diag.py > gpurun_out/diag/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; grep -E "RESULT|final" gpurun_out/diag/$n.log | head -8
  [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
  return 0
}
for v in ${DIAG_VARIANTS:-none_sync1_hist fake_hist}; do
  case $v in
    none_sync1_hist) run $v DIAG_COMM=none DIAG_SYNC=1 DIAG_STEPS=10 DIAG_HIST=1 || exit $? ;;
    fake_hist) run $v DIAG_COMM=fake DIAG_HIST=1 || exit $? ;;
    rccl) run $v DIAG_COMM=rccl || exit $? ;;
    fake) run $v DIAG_COMM=fake || exit $? ;;
    nomiopen) run $v DIAG_COMM=none DIAG_SYNC=1 DIAG_STEPS=30 DIAG_NOMIOPEN=1 || exit $? ;;
    noempty) run $v DIAG_COMM=none DIAG_SYNC=1 DIAG_STEPS=30 DIAG_NOEMPTY=1 || exit $? ;;
    noempty_fake) run $v DIAG_COMM=fake DIAG_NOEMPTY=1 || exit $? ;;
    nomiopen_fake) run $v DIAG_COMM=fake DIAG_NOMIOPEN=1 || exit $? ;;
    none_sync1) run $v DIAG_COMM=none DIAG_SYNC=1 DIAG_STEPS=30 || exit $? ;;
  esac
done
