#!/bin/bash
# Round-end evidence in one GPU call: smoke + GPU tests + bench + trace
# (gpu_check.sh), the C2 profile set (round_profile.sh), and the C4 bench with
# its kernel trace.  Each step has its own time limit; a fatal status stops it.
set -u
TAG=${TAG:-ev} bash tools/gpu_check.sh || exit $?
TAG=${TAG:-ev}_prof bash tools/round_profile.sh || exit $?
OUT=gpurun_out/${TAG:-ev}_c4; mkdir -p $OUT
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --host-otlp-spans 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
rc=$?; echo "bench c4 rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/trace" -o run \
   -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --host-otlp-spans 0 --streams 1 > "$GRAFT_REPO_ROOT/$OUT/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/trace.err"
echo "trace c4 rc=$?" >> "$GRAFT_REPO_ROOT/$OUT/status.txt"
