#!/bin/bash
# PMC passes for the ingest kernel variants: TAG=x VARS="8 0" FLAGS="0 31" tools/pmc2.sh
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
run() {  # $1 = label, rest = counters
  local label=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$label" -o run \
      -- python3 "$GRAFT_REPO_ROOT/tools/prof_driver.py" > "$OUT/$label.log" 2>&1
  local rc=$?
  echo "$label rc=$rc" >> "$OUT/status.txt"
  case $rc in 0|1|2) return 0 ;; *) echo "FATAL $rc" >> "$OUT/status.txt"; exit $rc ;; esac
}
for V in ${VARS:-8}; do for F in ${FLAGS:-0}; do
  export SPANAGG_VARIANT=$V PROF_FLAGS=$F PROF_REPS=3
  run "v$V.f$F.A" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
  run "v$V.f$F.B" SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
  run "v$V.f$F.C" FETCH_SIZE GRBM_GUI_ACTIVE
done; done
echo done >> "$OUT/status.txt"
