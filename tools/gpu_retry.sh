#!/bin/bash
# usage: gpu_retry.sh LOG TIMEOUT CMD — retries only when gpurun reports rc 3 (no box / slot:
# nothing ran, nothing charged)
LOG=$1; TO=$2; shift 2
for t in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "rc=$rc attempt=$t" >> $LOG; exit $rc; fi
  sleep 90
done
echo "gave up" >> $LOG
