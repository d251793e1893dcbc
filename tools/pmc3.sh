#!/bin/bash
# memory-pipeline / issue counters for the ingest kernel: TAG=x VARS="8" tools/pmc3.sh
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
run() {
  local label=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$label" -o run \
      -- python3 "$GRAFT_REPO_ROOT/tools/prof_driver.py" > "$OUT/$label.log" 2>&1
  local rc=$?
  echo "$label rc=$rc" >> "$OUT/status.txt"
  case $rc in 0|1|2) return 0 ;; *) echo "FATAL $rc" >> "$OUT/status.txt"; exit $rc ;; esac
}
for V in ${VARS:-8}; do
  export SPANAGG_VARIANT=$V PROF_FLAGS=${PROF_FLAGS:-0} PROF_REPS=3
  run "v$V.D" SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU
  run "v$V.E" SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_THREAD_CYCLES_VALU SQ_IFETCH SQ_INST_LEVEL_VMEM SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH
  run "v$V.F" TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
  run "v$V.G" TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum GRBM_GUI_ACTIVE
done
echo done >> "$OUT/status.txt"
