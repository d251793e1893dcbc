# Scatter occupancy A/B on one box: default (2,048 bins x 4-record stages,
# one 1,024-thread workgroup per CU) vs 1,024 bins x 4-record stages (76 KiB
# LDS) with VGPRs capped at 64 so two workgroups share a CU (grid 512), with
# 4 and 2 spans per thread per round; parity first.
set -u
OUT=gpurun_out/${TAG:-c4o}; mkdir -p $OUT
run_par() {  # name lib
  SPANAGG_LIB=$2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or high_card or partitioned" > $OUT/pytest_$1.log 2>&1
  rc=$?; echo "pytest $1 rc=$rc" >> $OUT/status.txt; return $rc
}
L=$PWD/tools/old
run_par b10s4w8 $L/libspanagg_b10s4w8.so || exit 1
run_par b10s4w8u2 $L/libspanagg_b10s4w8u2.so || exit 1
run_par b11s2 $L/libspanagg_b11s2.so || exit 1
abl() {  # name lib grid
  SPANAGG_LIB=$2 SPANAGG_PART_GRID=$3 ABL_WORKLOAD=c4 ABL_FLAGS="full:0" ABL_VARS="" ABL_REPS=5 ABL_ROUNDS=3 timeout -k 10 200 python tools/ablate.py > $OUT/abl_$1_$r.json 2> $OUT/abl_$1.err
  rc=$?; echo "abl $1 $r rc=$rc" >> $OUT/status.txt; return $rc
}
for r in 1 2; do
  abl base $PWD/opentelemetry-demo_amd/spanagg/libspanagg.so 256 || exit 1
  abl b10s4w8_g512 $L/libspanagg_b10s4w8.so 512 || exit 1
  abl b10s4w8u2_g512 $L/libspanagg_b10s4w8u2.so 512 || exit 1
  abl b10s4_g256 $L/libspanagg_b10s4.so 256 || exit 1
  abl b11s2_g256 $L/libspanagg_b11s2.so 256 || exit 1
done
