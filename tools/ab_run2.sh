# two-stream overlap check: GPU parity (full), bench at 1 and 2 streams, kernel trace of 2 streams
set -u
OUT=gpurun_out/${TAG:-ab2}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
for S in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --host-otlp-spans 0 --streams $S > $OUT/bench_s$S.json 2> $OUT/bench_s$S.err
  rc=$?; echo "bench s$S rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
done
SPANAGG_VARIANT=16 timeout -k 10 200 python bench.py --no-cpu-baseline --host-otlp-spans 0 --streams 2 > $OUT/bench_v16_s2.json 2> $OUT/bench_v16.err
echo "bench v16 rc=$?" >> $OUT/status.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
   -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --host-otlp-spans 0 > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"
echo "prof rc=$?" >> $GRAFT_REPO_ROOT/$OUT/status.txt
