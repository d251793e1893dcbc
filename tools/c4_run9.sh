# Same-box A/B: scatter fast path for used-up bin runs (default) vs without
# (tools/old/libspanagg_noskip.so, -DSA_PART_SKIP_USED=0); uniform and Zipf C4.
set -u
OUT=gpurun_out/${TAG:-c4s}; mkdir -p $OUT
for r in 1 2 3; do
  for v in skip noskip; do
    lib=$PWD/opentelemetry-demo_amd/spanagg/libspanagg.so; [ $v = noskip ] && lib=$PWD/tools/old/libspanagg_noskip.so
    for w in c4 c4zipf; do
      SPANAGG_LIB=$lib timeout -k 10 200 python bench.py --workload $w --steps 20 --no-cpu-baseline --host-otlp-spans 0 --h2d-reps 0 > $OUT/${v}_${w}_$r.json 2> $OUT/${v}_${w}.err || exit 1
    done
  done
done
