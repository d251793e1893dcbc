#!/bin/bash
# rocprofv3 kernel-trace stats of the C4 benches (uniform and Zipf mixes) on
# the current build.  usage: bash tools/c4_trace.sh
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/c4trace; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for w in c4 c4zipf; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$w" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload $w --steps 20 --warmup 3 --no-cpu-baseline \
       --host-otlp-spans 0 --h2d-reps 0 > "$OUT/${w}_bench.json" 2> "$OUT/${w}.err" || exit $?
done
