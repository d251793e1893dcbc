# Overflow-table size A/B on one box: default (4-record stages, 64 entries)
# vs 2-record stages with 256 / 512 entries; uniform and Zipf C4; parity first.
set -u
OUT=gpurun_out/${TAG:-c4h}; mkdir -p $OUT
L=$PWD/tools/old
for v in s2h8 s2h9; do
  SPANAGG_LIB=$L/libspanagg_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or high_card or partitioned or c4_full" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit 1
done
for r in 1 2; do
  for v in base s2h8 s2h9; do
    lib=$L/libspanagg_$v.so; [ $v = base ] && lib=$PWD/opentelemetry-demo_amd/spanagg/libspanagg.so
    for w in c4 c4zipf; do
      SPANAGG_LIB=$lib timeout -k 10 200 python bench.py --workload $w --steps 20 --no-cpu-baseline --host-otlp-spans 0 --h2d-reps 0 > $OUT/${v}_${w}_$r.json 2> $OUT/${v}_${w}.err
      rc=$?; echo "$v $w $r rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit 1
    done
  done
done
