# same-box A/B: slab sets x streams x variant
set -u
OUT=gpurun_out/${TAG:-ab4}; mkdir -p $OUT
B="python bench.py --no-cpu-baseline --host-otlp-spans 0"
for r in 1 2; do
  for V in 14 16; do for N in 1 2 3 4; do for S in 1 2; do
    SPANAGG_VARIANT=$V SPANAGG_SLAB_SETS=$N timeout -k 10 200 $B --streams $S > $OUT/v${V}_n${N}_s${S}_$r.json 2>/dev/null || exit $?
  done; done; done
  echo "round $r ok" >> $OUT/status.txt
done
