#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel
# trace. Each GPU step has its own time limit; a fault, abort, segfault or
# timeout ends the script (no further GPU work in the same call).
set -u
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = rc, $2 = step
  case "$1" in
    0|1|2) return 0 ;;   # ok / test failures / usage
    *) echo "FATAL rc=$1 in $2; stopping" | tee -a "$OUT/status.txt"; exit "$1" ;;
  esac
}
rocminfo 2>/dev/null | grep -m1 -E "gfx950" > "$OUT/device.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/status.txt"; stop_if_fatal $rc smoke
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/status.txt"; stop_if_fatal $rc pytest
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/status.txt"; stop_if_fatal $rc bench
if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"
  rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof rc=$rc" | tee -a "$OUT/status.txt"; stop_if_fatal $rc rocprof
fi
echo done | tee -a "$OUT/status.txt"
