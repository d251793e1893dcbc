#!/bin/bash
# gpurun wrapper: retries ONLY when gpurun reports a transient box-preparation
# failure (nothing ran, nothing charged). Any run that started is never retried.
# usage: tools/gpu.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient"; then
    sleep $((30 * i)); continue
  fi
  exit $rc
done
exit 3
