#!/bin/bash
# Round-4: one-step kernel timelines of the rank-share step (rank 0 of 8) under the inverse schedules.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for v in "p0:LVAE_CI_PIPE=0" "p2:LVAE_CI_PAIR=0"; do
  n=${v%%:*}; e=${v#*:}
  env $e NAME=s8_$n bash scripts/trace_step.sh --rank-share 8 || exit 1
done
