#!/bin/bash
set -u
OUT=gpurun_out/${TAG:-it}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/status.txt"; case $2 in 0|1) ;; *) echo FATAL >> "$OUT/status.txt"; exit $2 ;; esac; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; st pytest $?
timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/vc2.json" 2> "$OUT/c2.err"; st c2 $?
timeout -k 10 300 python bench.py --no-cpu-baseline --workload c4 --steps 10 --warmup 2 > "$OUT/vc4.json" 2> "$OUT/c4.err"; st c4 $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/kt" -o run -- python3 "$GRAFT_REPO_ROOT/tools/prof_driver.py" > "$GRAFT_REPO_ROOT/$OUT/kt.log" 2>&1; cd "$GRAFT_REPO_ROOT"; st ktrace $?
echo done >> "$OUT/status.txt"
