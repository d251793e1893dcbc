# C4 partitioned path ablation: median us per 10M-span launch per engine variant
set -u
OUT=gpurun_out/${TAG:-c4abl}; mkdir -p $OUT
ABL_WORKLOAD=c4 ABL_FLAGS="${ABL_FLAGS:-full:0,no_flush:8,no_red:1,no_hll:2}" ABL_VARS="" ABL_REPS=5 ABL_ROUNDS=3 timeout -k 10 400 python tools/ablate.py > $OUT/abl.json 2> $OUT/abl.err
echo "abl rc=$?" >> $OUT/status.txt
SPANAGG_HBM_PART=0 ABL_WORKLOAD=c4 ABL_FLAGS="atomic_full:0" ABL_VARS="" ABL_REPS=5 ABL_ROUNDS=3 timeout -k 10 400 python tools/ablate.py > $OUT/abl_atomic.json 2> $OUT/abl_atomic.err
echo "abl atomic rc=$?" >> $OUT/status.txt
