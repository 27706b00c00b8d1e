#!/bin/bash
# gpurun, waiting while no box is free (the call did not run: nothing charged); honours the
# "retry in Ns" the client prints
# usage: tools/gpq.sh LOG TIMEOUT CMD
LOG=$1; TO=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if ! grep -q "no free box right now\|backing off\|status=transient" $LOG; then echo "rc=$rc"; tail -5 $LOG; exit $rc; fi
  w=$(grep -o "retry in [0-9]*s" $LOG | tail -1 | grep -o "[0-9]*")
  sleep $(( ${w:-120} + 15 ))
done
echo "gave up"; exit 3
