#!/bin/bash
# run one gpurun command, retrying ONLY when the pool had no box / slot (nothing
# ran, nothing charged): at most 8 attempts, 4 minutes apart.  Output -> $OUT.
OUT=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout ${GPU_TIMEOUT:-900} -- "$@" > $OUT 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" $OUT; then
    echo "attempt $i: no box ($rc)" >> $OUT.retries
    sleep 240
    continue
  fi
  exit $rc
done
exit 3
