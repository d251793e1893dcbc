set -u
OUT=gpurun_out/${TAG:-c4h}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or high_card or partitioned" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
for r in 1 2; do
for L in default u4 u8; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/tools/old/libspanagg_$L.so; fi
  SPANAGG_LIB=$LIB ABL_WORKLOAD=c4 ABL_FLAGS="full:0" ABL_VARS="" ABL_REPS=5 ABL_ROUNDS=3 timeout -k 10 400 python tools/ablate.py > $OUT/abl_${L}_$r.json 2> $OUT/abl_$L.err
  echo "abl $L rc=$?" >> $OUT/status.txt
done; done
