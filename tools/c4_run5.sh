# Partitioned path A/B on one box: GPU parity, then C4 launches of the current
# library against tools/old/libspanagg_prev.so (the previous commit's build).
set -u
OUT=gpurun_out/${TAG:-c4i}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
for r in 1 2; do
  ABL_WORKLOAD=c4 ABL_FLAGS="full:0" ABL_VARS="" ABL_REPS=5 ABL_ROUNDS=3 timeout -k 10 400 python tools/ablate.py > $OUT/abl_$r.json 2> $OUT/abl.err
  echo "abl rc=$?" >> $OUT/status.txt
  SPANAGG_LIB=$PWD/tools/old/libspanagg_prev.so ABL_WORKLOAD=c4 ABL_FLAGS="full:0" ABL_VARS="" ABL_REPS=5 ABL_ROUNDS=3 timeout -k 10 400 python tools/ablate.py > $OUT/abl_prev_$r.json 2> $OUT/abl_prev.err
  echo "abl prev rc=$?" >> $OUT/status.txt
done
