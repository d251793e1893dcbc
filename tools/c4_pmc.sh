# C4 HBM traffic per kernel: FETCH_SIZE and WRITE_SIZE in separate passes
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-c4pmc}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  PROF_WORKLOAD=c4 timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -o run \
    -- python3 "$GRAFT_REPO_ROOT/tools/prof_driver.py" > "$OUT/$C.log" 2>&1
  rc=$?; echo "$C rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
done
