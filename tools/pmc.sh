#!/bin/bash
# PMC passes for the ingest kernel (one rocprofv3 --pmc pass per counter group;
# never combined with tracing domains).  usage: TAG=x LIBS="new old" tools/pmc.sh
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
run() {  # $1 = label, $2 = lib, rest = counters
  local label=$1 lib=$2; shift 2
  SPANAGG_LIB=$lib timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$label" -o run \
      -- python3 "$GRAFT_REPO_ROOT/tools/prof_driver.py" > "$OUT/$label.log" 2>&1
  local rc=$?
  echo "$label rc=$rc" >> "$OUT/status.txt"
  case $rc in 0|1|2) return 0 ;; *) echo "FATAL $rc" >> "$OUT/status.txt"; exit $rc ;; esac
}
for L in ${LIBS:-new}; do
  lib=$GRAFT_REPO_ROOT/opentelemetry-demo_amd/spanagg/libspanagg.so
  [ "$L" = old ] && lib=$GRAFT_REPO_ROOT/build/old/libspanagg.so
  run "$L.A" "$lib" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
  run "$L.B" "$lib" SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
  run "$L.C" "$lib" FETCH_SIZE GRBM_GUI_ACTIVE
  run "$L.D" "$lib" WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
done
echo done >> "$OUT/status.txt"
