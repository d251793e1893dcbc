set -u
OUT=gpurun_out/${TAG:-c4g}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
SPANAGG_PART_STAGE=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or high_card or partitioned" > $OUT/pytest_nostage.log 2>&1
rc=$?; echo "pytest nostage rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
ABL_FLAGS="full:0,no_flush:8,no_red:1" bash tools/c4_abl.sh
SPANAGG_PART_STAGE=0 ABL_WORKLOAD=c4 ABL_FLAGS="nostage_full:0" ABL_VARS="" ABL_REPS=5 ABL_ROUNDS=3 timeout -k 10 400 python tools/ablate.py > $OUT/abl_nostage.json 2> $OUT/abl_nostage.err
echo "abl nostage rc=$?" >> $OUT/status.txt
