#!/bin/bash
# Round evidence on one GPU box: bench (with CPU baseline), rocprofv3 kernel-trace
# stats of a shorter bench run, and FETCH_SIZE / WRITE_SIZE PMC passes (separate,
# no tracing domains).  usage: TAG=r1 bash tools/round_profile.sh
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
st() { echo "$1 rc=$2" >> "$OUT/status.txt"; case $2 in 0|1|2) ;; *) echo FATAL >> "$OUT/status.txt"; exit $2 ;; esac; }
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"; st bench $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --host-otlp-spans 0 > "$OUT/trace_bench.json" 2> "$OUT/trace.err"; st trace $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_s1" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --host-otlp-spans 0 --streams 1 > "$OUT/trace_s1_bench.json" 2> "$OUT/trace_s1.err"; st trace_s1 $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run \
  -- python3 "$GRAFT_REPO_ROOT/tools/prof_driver.py" > "$OUT/pmc_fetch.log" 2>&1; st pmc_fetch $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run \
  -- python3 "$GRAFT_REPO_ROOT/tools/prof_driver.py" > "$OUT/pmc_write.log" 2>&1; st pmc_write $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$OUT/pmc_lds" -o run \
  -- python3 "$GRAFT_REPO_ROOT/tools/prof_driver.py" > "$OUT/pmc_lds.log" 2>&1; st pmc_lds $?
echo done >> "$OUT/status.txt"
