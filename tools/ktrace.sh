#!/bin/bash
# kernel-trace stats of prof_driver under given flags/variants: TAG=x CASES="8:0 8:264" tools/ktrace.sh
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-kt}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in ${CASES:-8:0}; do
  V=${C%%:*}; F=${C##*:}
  SPANAGG_VARIANT=$V PROF_FLAGS=$F PROF_REPS=${PROF_REPS:-6} timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/v$V.f$F" -o run \
    -- python3 "$GRAFT_REPO_ROOT/tools/prof_driver.py" > "$OUT/v$V.f$F.log" 2>&1
  rc=$?; echo "v$V.f$F rc=$rc" >> "$OUT/status.txt"
  case $rc in 0|1|2) ;; *) echo FATAL >> "$OUT/status.txt"; exit $rc ;; esac
done
echo done >> "$OUT/status.txt"
