# same-box A/B: previous commit's library (tools/old) vs the current one
set -u
OUT=gpurun_out/${TAG:-ab3}; mkdir -p $OUT
B="python bench.py --no-cpu-baseline --host-otlp-spans 0"
for r in 1 2; do
  timeout -k 10 200 $B --streams 1 > $OUT/new_s1_$r.json 2>/dev/null || exit $?
  SPANAGG_LIB=$PWD/tools/old/libspanagg_head.so timeout -k 10 200 $B --streams 1 > $OUT/old_s1_$r.json 2>/dev/null || exit $?
  timeout -k 10 200 $B --streams 2 > $OUT/new_s2_$r.json 2>/dev/null || exit $?
  SPANAGG_VARIANT=16 timeout -k 10 200 $B --streams 2 > $OUT/v16_s2_$r.json 2>/dev/null || exit $?
  SPANAGG_VARIANT=16 timeout -k 10 200 $B --streams 1 > $OUT/v16_s1_$r.json 2>/dev/null || exit $?
  echo "round $r ok" >> $OUT/status.txt
done
