#!/bin/bash
# (run from the build container: tools/gpuq.sh LOG [gpurun args] -- CMD)
# queue a gpurun call: retries ONLY when the pool had no free box / slot (exit 3: nothing ran)
log=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1; rc=$?
  [ $rc -ne 3 ] && break
  sleep 90
done
echo "EXIT $rc" >> "$log"
