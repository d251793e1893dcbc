#!/bin/bash
# bench.py (no CPU baseline) under several kernel variants: VARS="0 8" tools/bench_vars.sh
set -u
OUT=gpurun_out/${TAG:-bv}
mkdir -p "$OUT"
for V in ${VARS:-8}; do
  SPANAGG_VARIANT=$V timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/v$V.json" 2> "$OUT/v$V.err"
  rc=$?; echo "v$V rc=$rc" >> "$OUT/status.txt"
  case $rc in 0|1) ;; *) echo FATAL >> "$OUT/status.txt"; exit $rc ;; esac
done
echo done >> "$OUT/status.txt"
