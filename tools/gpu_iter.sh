#!/bin/bash
# one iteration: GPU parity (default variant), then bench under several variants
set -u
OUT=gpurun_out/${TAG:-it}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; case $rc in 0|1) ;; *) echo FATAL >> "$OUT/status.txt"; exit $rc ;; esac
for V in ${VARS:-}; do
  SPANAGG_VARIANT=$V timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/v$V.json" 2> "$OUT/v$V.err"
  rc=$?; echo "bench v$V rc=$rc" >> "$OUT/status.txt"; case $rc in 0|1) ;; *) echo FATAL >> "$OUT/status.txt"; exit $rc ;; esac
done
echo done >> "$OUT/status.txt"
