set -u
OUT=gpurun_out/ab1; mkdir -p $OUT
for V in 16 17 18; do
  SPANAGG_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_v$V.log 2>&1
  rc=$?; echo "pytest v$V rc=$rc" >> $OUT/status.txt
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
ABL_NO_DIAG=1 ABL_VARS=14,16,17,18 ABL_REPS=10 timeout -k 10 300 python tools/ablate.py > $OUT/ab.json 2> $OUT/ab.err
echo "ab rc=$?" >> $OUT/status.txt
