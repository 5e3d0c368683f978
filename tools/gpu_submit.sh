#!/bin/bash
# Submit one gpurun call; when no box is free (exit 3, or a transient failure before the command
# ran) wait and submit again, at most TRIES times. A call whose command ran is never repeated.
# usage: tools/gpu_submit.sh LOG TIMEOUT 'command'
LOG=$1; T=$2; CMD=$3
for i in $(seq 1 ${TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$CMD" > $LOG 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient rc=None" $LOG; then
    echo "[submit] try $i: no box ($rc)" >> $LOG.tries; sleep ${WAIT:-150}; continue
  fi
  echo "[submit] done rc=$rc" >> $LOG.tries; exit $rc
done
