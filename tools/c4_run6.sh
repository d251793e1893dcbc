# Partition geometry A/B on one box: 2,048 bins x 4-record stages (current)
# vs 1,024 bins x 8-record stages (tools/old/libspanagg_b10.so); parity first.
set -u
OUT=gpurun_out/${TAG:-c4l}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or high_card or partitioned" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
SPANAGG_LIB=$PWD/tools/old/libspanagg_b10.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or high_card or partitioned" > $OUT/pytest_b10.log 2>&1
rc=$?; echo "pytest b10 rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
for r in 1 2; do
  ABL_WORKLOAD=c4 ABL_FLAGS="full:0" ABL_VARS="" ABL_REPS=5 ABL_ROUNDS=3 timeout -k 10 400 python tools/ablate.py > $OUT/abl_b11_$r.json 2> $OUT/abl.err
  echo "abl b11 rc=$?" >> $OUT/status.txt
  SPANAGG_LIB=$PWD/tools/old/libspanagg_b10.so ABL_WORKLOAD=c4 ABL_FLAGS="full:0" ABL_VARS="" ABL_REPS=5 ABL_ROUNDS=3 timeout -k 10 400 python tools/ablate.py > $OUT/abl_b10_$r.json 2> $OUT/abl_b10.err
  echo "abl b10 rc=$?" >> $OUT/status.txt
done
