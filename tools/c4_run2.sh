set -u
OUT=gpurun_out/${TAG:-c4d}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; case $rc in 0|1) ;; *) exit $rc ;; esac
ABL_FLAGS="full:0,no_flush:8,no_red:1" bash tools/c4_abl.sh
timeout -k 10 300 python bench.py --no-cpu-baseline --host-otlp-spans 0 > $OUT/c2.json 2>/dev/null
echo "c2 rc=$?" >> $OUT/status.txt
