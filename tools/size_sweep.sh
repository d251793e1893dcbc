#!/bin/bash
# Kernel time vs batch size (fixed cost per launch = intercept):
#   SIZES="1000000 5000000 10000000" tools/size_sweep.sh
set -u
OUT=gpurun_out/${TAG:-sweep}
mkdir -p "$OUT"
for N in ${SIZES:-1000000 2500000 5000000 10000000 15000000}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --spans "$N" --steps 30 --warmup 3 > "$OUT/n$N.json" 2> "$OUT/n$N.err"
  rc=$?; echo "n$N rc=$rc" >> "$OUT/status.txt"
  case $rc in 0|1) ;; *) echo FATAL >> "$OUT/status.txt"; exit $rc ;; esac
done
echo done >> "$OUT/status.txt"
