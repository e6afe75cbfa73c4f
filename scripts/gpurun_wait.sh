#!/bin/bash
# gpurun_wait.sh LOG CMD: submit CMD through gpurun, resubmitting ONLY while the pool answers rc=3 (no
# box / slot free: nothing ran, nothing charged) or a transient back-off; any other outcome ends it.
LOG=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout ${GPURUN_TIMEOUT:-1200} -- "$@" > $LOG 2>&1
  rc=$?
  echo "rc=$rc (attempt $i)" >> $LOG
  if [ $rc -ne 3 ]; then exit $rc; fi
  w=$(grep -o "retry in [0-9]*s" $LOG | grep -o "[0-9]*" | head -1)
  sleep $(( ${w:-200} + 20 ))
done
exit 3
