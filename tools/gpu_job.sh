#!/bin/bash
# One GPU-box job made of named steps, each under its own time limit.
#   usage (inside gpurun): TAG=name bash tools/gpu_job.sh STEP [STEP ...]
# Steps:
#   smoke            __graft_entry__.smoke() (one small hot-path run vs the oracle)
#   tests            every -m gpu test (pytest, per-test timeout)
#   tests:<file>     one test file, e.g. tests:tests/test_gpu_binned.py
#   bench            the default bench line (C2 + C4 sub-objects, CPU baselines)
#   selflaunch_<n>   bare `bench.py --gpus n` (it spawns its n ranks), every rank on this GPU, gloo
#   rehearse_<n>     bench.py's n-rank path (torch.distributed.run) with every
#                    rank on this one GPU and gloo collectives (a rehearsal)
#   bench_<wl>       a short bench of one workload (c2, c4, c4zipf), no baselines
#   abvar_<a>_<b>..  C2 bench of laboratory-build kernel variants a, b, ... (3 rounds)
#   streams_<wl>     bench of <wl> with 1 and with 2 launch streams (2 rounds)
#   labtests_<v>     the small-table parity suites on laboratory-build variant v
#   libab_<wl>_<name>  bench of <wl> on the product library and on spanagg/lib<name>.so (3 rounds)
#   btpair_<wl>      bench of <wl> with binned aggregates in pairs / one per launch (3 rounds)
#   btagg_<wl>       bench of <wl> with 512- and 1,024-thread aggregate workgroups (2 rounds)
#   labbin_<KNOB=v>  the binned parity suites on the laboratory build with KNOB=v
#   hostprof_<t>     host_rate.js (GPU ingest, t threads) under node --cpu-prof
#   hostprofc4_<t>   the same over the C4 vocabulary (--highcard)
#   colab            colbench against host/node/build/$COL_OTHER (3 rounds, 16 and 8 threads)
#   colbench         the native columnizer alone (host/node/build/colbench) at 1-16 threads
#   labexpo_<KNOB=v> the exponential-histogram suites on the laboratory build with KNOB=v
#   xrec_<wl>        bench of <wl> with the expo slab path's span records on / off (3 rounds)
#   evscope_<wl>     bench of <wl> with the engine's events at device / system scope (2 rounds)
#   labtrace_<wl>_<VAR=v>  rocprofv3 trace of a 100-step bench of <wl> on the laboratory build with VAR=v
#   btpipe_<wl>      bench of <wl> with the binned launch pipeline on and off (2 rounds)
#   ablate_<wl>      tools/ablate.py over the ABL_FLAGS / ABL_ENVS variant set for <wl>
#   c2stamps         tools/stamps.py: per-workgroup phases of the C2 kernel (STAMP_VARS variants)
#   xcstamps[_<d>]   tools/xc_stamps.py: c2expo counting-kernel phases (_d: laboratory, SPANAGG_XC_DIAG=d)
#   stamps_<wl>      tools/bt_stamps.py: per-workgroup phase timeline (c4, c4zipf)
#   sweep            C2 kernel time vs batch size (SIZES="1000000 5000000 ...")
#   group_<wl>       rocprofv3 --kernel-trace --stats of bench.py --group 8 (an
#                    8-member group on this device: partition + group flush)
#   trace_<wl>       rocprofv3 --kernel-trace --stats of a short bench of <wl>
#   ptrace_<wl>      the same over a long timed region (PSTEPS, default 400 steps,
#                    one stream: overlapping launches would stretch each other's
#                    traced durations); the bench line is the last line of the log
#   pmc_<wl>_<set>   one rocprofv3 --pmc pass (set: fetch, write, lds, sq) over
#                    tools/prof_driver.py for <wl>
# Outputs go to gpurun_out/$TAG/.  Any failing step ends the job (exit code
# kept): a failed test may be a GPU fault, after which nothing more runs on
# the GPU in that call.  LENIENT=1 lets a step that returned 1 continue.
set -u
TAG=${TAG:-job}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOTDIR=$PWD

run() {  # name, seconds, command...
  local name=$1 t=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/status.txt"
  if [ "$rc" = 0 ] || { [ "$rc" = 1 ] && [ "${LENIENT:-0}" = 1 ]; }; then return 0; fi
  echo "FATAL $name rc=$rc" >> "$OUT/status.txt"
  exit $rc
}

BQ="--no-cpu-baseline --host-otlp-spans 0 --h2d-reps 0"
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    sweep) for N in ${SIZES:-1000000 2500000 5000000 10000000 15000000}; do
        run "sweep_n$N" 200 python bench.py --sub "" --spans "$N" --steps 30 --warmup 3 $BQ; done ;;
    c2stamps) STAMP_SETS=${STAMP_SETS:-full} STAMP_VARS=${STAMP_VARS:-20,21} run c2stamps 300 python tools/stamps.py ;;
    stamps_*) wl=${step#stamps_}; WL=$wl run "stamps_$wl" 300 python tools/bt_stamps.py ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    tests:*) f=${step#tests:}; run "tests_$(basename "$f" .py)" 600 python -u -m pytest "$f" -m gpu -x -v --timeout 300 --timeout-method thread ;;
    bench) run bench 500 python bench.py ;;
    rehearse_*) n=${step#rehearse_}; SPANAGG_BENCH_ONE_DEVICE=1 run "rehearse_n$n" 400 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus "$n" --steps 10 \
        --warmup 2 --settle 4 --soak-s 0 ;;
    selflaunch_*) n=${step#selflaunch_}; SPANAGG_BENCH_ONE_DEVICE=1 run "selflaunch_n$n" 400 python bench.py --gpus "$n" \
        --steps ${SL_STEPS:-20} --soak-s 0 ;;  # bench.py starts its own n ranks (no outer launcher), all on this GPU
    colbench) (cd host/node && node test/host_rate.js 2000000 --dump /tmp/req_plain.bin > /dev/null && \
        node test/host_rate.js 2000000 --events --dump /tmp/req_ev.bin > /dev/null) || exit 1
      for t in ${COL_THREADS:-1 4 8 16}; do run "colbench_t$t" 120 host/node/build/colbench /tmp/req_plain.bin --threads "$t"; done
      run colbench_ex_t16 120 host/node/build/colbench /tmp/req_ev.bin --threads 16 --exemplars --events ;;
    colabhc) (cd host/node && node test/host_rate.js 2000000 --highcard --dump /tmp/req_hc.bin > /dev/null) || exit 1  # C4 vocabulary, http.route dimension
      for r in 1 2 3; do for b in colbench ${COL_OTHER:-colbench_olddim}; do
        run "colabhc_${b}_r$r" 120 host/node/build/$b /tmp/req_hc.bin --threads 16 --dim http.route; done; done ;;
    colabex) (cd host/node && node test/host_rate.js 2000000 --events --dump /tmp/req_ev.bin > /dev/null) || exit 1  # exemplars + events
      for r in 1 2 3; do for b in colbench ${COL_OTHER:-colbench_olddim}; do
        run "colabex_${b}_r$r" 120 host/node/build/$b /tmp/req_ev.bin --threads 16 --exemplars --events; done; done ;;
    colab) (cd host/node && node test/host_rate.js 2000000 --dump /tmp/req_plain.bin > /dev/null) || exit 1  # colbench against build/colbench_<other>
      for r in 1 2 3; do for t in 16 8; do for b in colbench ${COL_OTHER:-colbench_condvar}; do
        run "colab_${b}_t${t}_r$r" 120 host/node/build/$b /tmp/req_plain.bin --threads "$t"; done; done; done ;;
    hostprof_*) t=${step#hostprof_}; run "hostprof_t$t" 200 node --cpu-prof --cpu-prof-dir="$OUT/hostprof_t$t" \
        --max-old-space-size=16000 host/node/test/host_rate.js 2000000 --gpu --threads "$t" --batch 128 ;;
    hostprofc4_*) t=${step#hostprofc4_}; run "hostprofc4_t$t" 300 node --cpu-prof --cpu-prof-dir="$OUT/hostprofc4_t$t" \
        --max-old-space-size=16000 host/node/test/host_rate.js 2000000 --gpu --threads "$t" --batch 128 --highcard ;;
    hostex_*) t=${step#hostex_}; run "hostex_t$t" 200 node --max-old-space-size=16000 host/node/test/host_rate.js 2000000 --gpu --threads "$t" --batch 128 --exemplars --events ;;
    hostc4_*) t=${step#hostc4_}; run "hostc4_t$t" 200 node --max-old-space-size=16000 host/node/test/host_rate.js 2000000 --gpu --threads "$t" --batch 128 --highcard ;;
    host_*) t=${step#host_}; run "host_t$t" 200 node --max-old-space-size=16000 host/node/test/host_rate.js 2000000 --gpu --threads "$t" --batch 128 ;;
    bench_*) wl=${step#bench_}; run "bench_$wl" 300 python bench.py --workload "$wl" --sub "" --steps 20 $BQ ;;
    abvar_*) vs=${step#abvar_}  # A/B of small-table kernel variants (laboratory build), rounds interleaved
      for r in 1 2 3; do for v in ${vs//_/ }; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_VARIANT=$v \
          run "abvar_v${v}_r$r" 200 python bench.py --workload c2 --sub "" --steps 50 --soak-s 0 --no-filter-off $BQ
      done; done ;;
    abhalf_*) rest=${step#abhalf_}; nps=${rest%%_*}; vs=${rest#*_}; [ "$vs" = "$rest" ] && vs=15_25
      # small-table variants (default 15 against 25, 512-thread workgroups) on a C2 vocabulary of 20 x nps names
      for r in 1 2 3; do for v in ${vs//_/ }; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_VARIANT=$v \
          run "abhalf${nps}_v${v}_r$r" 200 python bench.py --workload c2 --sub "" --steps 50 --soak-s 0 --no-filter-off \
          --names-per-service "$nps" $BQ
      done; done ;;
    btpipe_*) wl=${step#btpipe_}  # the binned launch pipeline on / off (laboratory build), rounds interleaved
      for r in 1 2; do for pp in 1 0; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_BT_PIPE=$pp \
          run "btpipe_${wl}_p${pp}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 40 --soak-s 0 --no-filter-off $BQ
      done; done ;;
    libab_*) rest=${step#libab_}; wl=${rest%%_*}; other=${rest#*_}  # product library against spanagg/lib<other>.so, e.g. libab_c2_spanagg_prediet
      for r in 1 2 3; do for lib in libspanagg "lib$other"; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/$lib.so \
          run "libab_${wl}_${lib}$([ "$lib" = libspanagg ] && echo "_vs_$other")_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 50 --soak-s 0 --no-filter-off \
          ${NPS:+--names-per-service $NPS} $BQ
      done; done ;;
    btpair_*) wl=${step#btpair_}  # binned launches aggregated in pairs / alone (laboratory build), rounds interleaved
      for r in 1 2 3; do for pp in 1 0; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_BT_PAIR=$pp \
          run "btpair_${wl}_p${pp}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 40 --soak-s 0 --no-filter-off $BQ
      done; done ;;
    btagg_*) wl=${step#btagg_}  # aggregate workgroups of 512 / 1,024 threads (laboratory build), rounds interleaved
      for r in 1 2; do for bb in 512 1024; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_BT_AGG_BLOCK=$bb \
          run "btagg_${wl}_b${bb}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 40 --soak-s 0 --no-filter-off $BQ
      done; done ;;
    labbin_*) knob=${step#labbin_}  # the binned parity suite on the laboratory build with one knob, e.g. labbin_SPANAGG_BT_AGG_BLOCK=1024
      (export SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so; export "$knob"; \
       run "labbin_${knob//=/}" 600 python -u -m pytest tests/test_gpu_binned.py "tests/test_gpu_regime.py" -m gpu -x -v \
         --timeout 300 --timeout-method thread) || exit $? ;;
    expoab_*) wl=${step#expoab_}  # c2expo: span records x slab sets (laboratory build), rounds interleaved
      for r in 1 2; do for x in 0 1; do for ns in 1 2; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_XREC=$x SPANAGG_SLAB_SETS=$ns \
          run "expoab_${wl}_x${x}_s${ns}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 40 --soak-s 0 --no-filter-off $BQ
      done; done; done ;;
    exposets_*) wl=${step#exposets_}  # c2expo with 1 / 2 / 3 slab sets (laboratory build), rounds interleaved
      for r in 1 2; do for ns in 1 2 3; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_SLAB_SETS=$ns \
          run "exposets_${wl}_s${ns}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 40 --soak-s 0 --no-filter-off $BQ
      done; done ;;
    xstream_*) wl=${step#xstream_}  # c2expo histogram kernels on an engine stream (1) / the caller's stream (0, product), laboratory build
      for r in 1 2 3; do for x in 1 0; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_XSTREAM=$x \
          run "xstream_${wl}_x${x}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 40 --soak-s 0 --no-filter-off $BQ
      done; done ;;
    xrectrace_*) wl=${step#xrectrace_}  # per-kernel trace of c2expo with span words 0 / 2 (laboratory build)
      for r in 1 2; do for x in 0 2; do
        (cd /tmp && SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_XREC=$x run "xrectrace_${wl}_x${x}_r$r" 200 \
          rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/xrectrace_${wl}_x${x}_r$r" -o run \
          -- python3 "$ROOTDIR/bench.py" --workload "$wl" --sub "" --steps 100 --streams 1 --soak-s 0 --no-filter-off ${XFC:-} $BQ) || exit $?
      done; done ;;
    xidxoff_*) wl=${step#xidxoff_}  # c2expo: the ingest kernel's bucket index work on / off (ablation, laboratory build)
      for r in 1 2; do for x in 0 1 2; do
        if [ $x != 0 ]; then export SPANAGG_XIDX_OFF=$x; else unset SPANAGG_XIDX_OFF; fi
        (cd /tmp && SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so run "xidxoff_${wl}_x${x}_r$r" 200 \
          rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/xidxoff_${wl}_x${x}_r$r" -o run \
          -- python3 "$ROOTDIR/bench.py" --workload "$wl" --sub "" --steps 100 --streams 1 --soak-s 0 --no-filter-off $BQ) || exit $?
      done; done; unset SPANAGG_XIDX_OFF ;;
    fresh_*) wl=${step#fresh_}  # every column fresh per launch (--fresh-cols) against trace ids only, rounds interleaved
      for r in 1 2; do for f in 0 1; do
        if [ $f = 1 ]; then fc=--fresh-cols; else fc=; fi
        run "fresh_${wl}_f${f}_r$r" 300 python bench.py --workload "$wl" --sub "" --steps 40 --soak-s 0 --no-filter-off $fc $BQ
      done; done ;;
    labexpo_*) knob=${step#labexpo_}  # the exponential-histogram suites on the laboratory build with one knob, e.g. labexpo_SPANAGG_XREC=0
      (export SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so; export "$knob"; \
       run "labexpo_${knob//=/}" 300 python -u -m pytest tests/test_gpu_expo.py tests/test_gpu_churn.py -m gpu -x -v \
         --timeout 300 --timeout-method thread) || exit $? ;;
    xrec_*) wl=${step#xrec_}  # exponential slab path: index records (2) / span records (1) / slots + times (0), laboratory build, rounds interleaved
      for r in 1 2 3; do for x in 2 1 0; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_XREC=$x \
          run "xrec_${wl}_x${x}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 40 --soak-s 0 --no-filter-off $BQ
      done; done ;;
    evscope_*) wl=${step#evscope_}  # engine events at device scope (default) / system scope (laboratory build)
      for r in 1 2; do for es in 0 1; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_EV_SYS=$es \
          run "evscope_${wl}_sys${es}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 50 --soak-s 0 --no-filter-off $BQ
      done; done ;;
    labtests_*) v=${step#labtests_}  # small-table parity suites on a laboratory-build variant
      SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_VARIANT=$v \
        run "labtests_v$v" 600 python -u -m pytest tests/test_gpu_parity.py tests/test_c5_windows.py tests/test_gpu_churn.py \
        "tests/test_gpu_regime.py::test_c2_bench_regime_40_variants_bit_exact" -m gpu -x -v --timeout 300 --timeout-method thread ;;
    streams_*) wl=${step#streams_}  # one launch stream against two, rounds interleaved
      for r in 1 2; do for n in 1 2; do
        run "streams_${wl}_s${n}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 50 --streams $n --soak-s 0 --no-filter-off $BQ
      done; done ;;
    ablate_*) wl=${step#ablate_}; ABL_WORKLOAD=$wl ABL_VARS=${ABL_VARS:-} run "ablate_$wl" 400 python tools/ablate.py ;;
    ptrace_*) wl=${step#ptrace_}  # the rocprofv3 summary the bench line's kernel_ms is checked against:
      # a long timed region so the cold and settling launches weigh little in the average
      (cd /tmp && run "ptrace_$wl" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ptrace_$wl" -o run \
         -- python3 "$ROOTDIR/bench.py" --workload "$wl" --sub "" --steps ${PSTEPS:-400} --streams 1 --soak-s 0 \
         --no-filter-off $BQ) || exit $? ;;
    kab_*) rest=${step#kab_}; wl=${rest%%_*}; lib=${rest#*_}  # ptrace of <wl> on spanagg/lib<lib>.so (per-kernel times of a variant)
      (cd /tmp && SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/lib$lib.so run "kab_${wl}_$lib" 300 rocprofv3 --kernel-trace --stats \
         --output-format csv -d "$OUT/kab_${wl}_$lib" -o run -- python3 "$ROOTDIR/bench.py" --workload "$wl" --sub "" \
         --steps ${PSTEPS:-200} --streams 1 --soak-s 0 --no-filter-off $BQ) || exit $? ;;
    group_*) wl=${step#group_}  # an 8-member group on this device: partition kernels + group flush
      (cd /tmp && run "group_$wl" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/group_$wl" -o run \
         -- python3 "$ROOTDIR/bench.py" --workload "$wl" --sub "" --group 8 --steps 20 --warmup 3 --soak-s 0 \
         --no-filter-off $BQ) || exit $? ;;
    labtrace_*) rest=${step#labtrace_}; wl=${rest%%_*}; knob=${rest#*_}  # e.g. labtrace_c4_SPANAGG_BT_PIPE=0
      (export SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so; export "$knob"; cd /tmp && \
       run "labtrace_${wl}_${knob//=/}" 300 rocprofv3 --kernel-trace --stats --output-format csv \
         -d "$OUT/labtrace_${wl}_${knob//=/}" -o run \
         -- python3 "$ROOTDIR/bench.py" --workload "$wl" --sub "" --steps 100 --streams 1 --soak-s 0 --no-filter-off $BQ) || exit $? ;;
    setev_*) wl=${step#setev_}  # slab-set event per launch on / off (laboratory build, one stream), rounds interleaved
      for r in 1 2; do for ne in 0 1; do
        if [ "$ne" = 1 ]; then export SPANAGG_NO_SETEV=1; else unset SPANAGG_NO_SETEV; fi
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so \
          run "setev_${wl}_ne${ne}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 50 --streams 1 --soak-s 0 --no-filter-off $BQ
      done; done; unset SPANAGG_NO_SETEV ;;
    trace2_*) wl=${step#trace2_}  # kernel trace of launches alternating over two streams (overlap or not)
      (cd /tmp && run "trace2_$wl" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace2_$wl" -o run \
         -- python3 "$ROOTDIR/bench.py" --workload "$wl" --sub "" --steps 100 --streams 2 --soak-s 0 --no-filter-off $BQ) || exit $? ;;
    xt_*) wl=${step#xt_}  # c2expo counting tail: LDS records + fold (1) / HBM atomics (0), laboratory build, rounds interleaved
      for r in 1 2; do for xt in 1 0; do
        SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_XT=$xt \
          run "xt_${wl}_x${xt}_r$r" 200 python bench.py --workload "$wl" --sub "" --steps 40 --soak-s 0 --no-filter-off $BQ
      done; done ;;
    xcstamps) run xcstamps 200 python tools/xc_stamps.py ;;  # c2expo counting-kernel phases (product build)
    xcstamps_*) d=${step#xcstamps_}  # the same on the laboratory build with SPANAGG_XC_DIAG=d (ablations)
      SPANAGG_LIB=$ROOTDIR/opentelemetry-demo_amd/spanagg/libspanagg_ab.so SPANAGG_XC_DIAG=$d \
        run "xcstamps_d$d" 200 python tools/xc_stamps.py ;;
    c4chunks) run c4chunks 200 "$ROOTDIR/build/c4_probe" 10000000 chunks ;;
    probe_*) p=${step#probe_}; run "probe_$p" 200 "$ROOTDIR/build/${p}_probe" ;;
    groupbench_*) wl=${step#groupbench_}  # an 8-member group on this device, no profiler (flush_ms as a caller sees it)
      run "groupbench_$wl" 300 python bench.py --workload "$wl" --sub "" --group 8 --steps 10 --warmup 2 --soak-s 0 \
         --no-filter-off $BQ ;;
    trace_*) wl=${step#trace_}
      (cd /tmp && run "trace_$wl" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$wl" -o run \
         -- python3 "$ROOTDIR/bench.py" --workload "$wl" --sub "" --steps 10 --warmup 2 --streams 1 --soak-s 0 --no-filter-off $BQ) || exit $? ;;
    pmc_*) rest=${step#pmc_}; wl=${rest%%_*}; set_=${rest#*_}
      case $set_ in
        fetch) ctr="FETCH_SIZE" ;;
        write) ctr="WRITE_SIZE" ;;
        lds) ctr="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES" ;;
        sq) ctr="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" ;;
        inst) ctr="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAVES" ;;
        act) ctr="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM" ;;
        ta) ctr="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" ;;
        *) echo "unknown pmc set $set_" >> "$OUT/status.txt"; exit 2 ;;
      esac
      (cd /tmp && PROF_WORKLOAD=$wl PROF_REPS=${PROF_REPS:-24} run "pmc_${wl}_$set_" 120 rocprofv3 --pmc $ctr --output-format csv \
         -d "$OUT/pmc_${wl}_$set_" -o run -- python3 "$ROOTDIR/tools/prof_driver.py") || exit $? ;;
    *) echo "unknown step $step" >> "$OUT/status.txt"; exit 2 ;;
  esac
done
echo done >> "$OUT/status.txt"
