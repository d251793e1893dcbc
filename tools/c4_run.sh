# partitioned HBM-table path: GPU parity on the HBM-path tests, then C4 bench part vs atomic
set -u
OUT=gpurun_out/${TAG:-c4}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "golden or high_card or partitioned or epoch or table_full or c2_small" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
for G in ${GRIDS:-256 512}; do
  SPANAGG_PART_GRID=$G timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --host-otlp-spans 0 --steps 20 --warmup 3 > $OUT/c4_part_g$G.json 2> $OUT/c4_part_g$G.err
  rc=$?; echo "part g$G rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
done
SPANAGG_HBM_PART=0 timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --host-otlp-spans 0 --steps 20 --warmup 3 > $OUT/c4_atomic.json 2> $OUT/c4_atomic.err
echo "atomic rc=$?" >> $OUT/status.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
   -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --host-otlp-spans 0 --streams 1 > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"
echo "prof rc=$?" >> $GRAFT_REPO_ROOT/$OUT/status.txt
