#!/bin/bash
# Submit one gpurun call, resubmitting only while the pool answers "no box / slot free" (exit 3:
# nothing ran, nothing charged).  Any other exit code ends it.  Usage: tools/gpurun_retry.sh LOG TIMEOUT CMD
LOG=$1; TO=$2; shift 2
for i in $(seq 1 20); do
    /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
    rc=$?
    [ $rc -ne 3 ] && exit $rc
    sleep 150
done
exit 3
