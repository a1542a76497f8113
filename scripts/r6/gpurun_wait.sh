#!/bin/bash
# retry only while gpurun reports "no slot" (rc 3: nothing ran, nothing charged)
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
exit 3
