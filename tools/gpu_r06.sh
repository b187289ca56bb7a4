#!/bin/bash
# Round-6 GPU session.  STEPS selects parts (default: tests bench); each GPU step has its own time limit and the
# script stops at the first failure.
#   tests     pytest -m gpu
#   smoke     __graft_entry__.smoke()
#   counters  tools/counters.py with the RT_COUNTERS=1 build tools/_var/cnt (events and lane utilisation per wave)
#   bench     the default bench line (N = 1)
#   rehearse  bench.py --gpus 2 --backend gloo (two ranks sharing the GPU; the c4 leg as a COPY group on rank 0)
#   trace     per-wave timeline of one c2 / c5 launch (tools/_var/trace, RT_WAVE_TRACE=2 build) with the attribution
#   c4n1      tools/c4_n1_probe.py: the one-rank rt_render_multi frame against plain c3 renders
#   hostw     tools/_mb_hostwrite (kernel stores into pinned host memory by store shape)
#   refill    tools/_var/mb_refill: traced wave durations replayed as sleeps, by LDS / VGPR footprint
#   abenv     tools/ab_env.py: context settings from the environment, one context each (ABENV_MODES)
#   sdma      tools/_var/mb_sdma: a frame's device-to-host copy on the SDMA engines vs the runtime's, beside a busy kernel
#   copyab    tools/copy_ab.py: draw()'s GRAY8 host frame by copy mode (COPY_SETTINGS mode:blocks, 3 = SDMA)
#   ab        tools/ab_libs.py over tools/_var/* (VARS=comma list, CONFIGS, ROUNDS; INFLIGHT for the bench pattern)
#   prof      one-stream rocprofv3 kernel-trace summaries at c2 / c3 / c5 (CONFIGS)
#   pmc       PMC passes per config (tools/pmc.sh)
#   mbunpack  tools/_mb_unpack (rank 0's GRAY8 -> RGBA8 expansion of a c4 frame against its HBM floors)
#   queues    tools/c4_gap_probe.py part 5, plain and under --kernel-trace (hardware queue of each stream kind)
#   c4probe   tools/c4_gap_probe.py (PARTS, NS, HBS)
#   count     tools/count.sh (PMC instruction counts per scene variant, VARIANTS)
#   profsdma  tools/prof_sdma.sh (kernel + memory-copy trace of the SDMA host-frame path)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
want() { case " ${STEPS:-tests bench} " in *" $1 "*) return 0;; esac; return 1; }
LIB=ray_tracer_fragment_shader_amd/lib/librt_amd.so
if want tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} \
      > "$OUT/gpu_tests.log" 2>&1
  rc=$?; cp "$OUT/gpu_tests.log" "$OUT/gpu_tests_$(date +%H%M%S).log"; tail -5 "$OUT/gpu_tests.log"
  [ $rc -eq 0 ] || { grep -n -i -A3 "memory access fault\|captured stderr" "$OUT/gpu_tests.log" | head -40; echo "pytest rc=$rc"; exit $rc; }
fi
if want smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
      || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 29; }
  tail -3 "$OUT/smoke.log"
fi
if want counters; then
  LIB=tools/_var/cnt/librt_amd.so timeout -k 10 300 python -u tools/counters.py ${CNT_CONFIGS:-c2,c3,c5} \
      > "$OUT/counters.jsonl" 2> "$OUT/counters.err" || { echo "counters failed"; tail -20 "$OUT/counters.err"; exit 30; }
  cat "$OUT/counters.jsonl"
fi
if want trace; then
  cp "$LIB" /tmp/librt_amd.base.so
  cp tools/_var/trace/librt_amd.so "$LIB"
  for c in ${TRACE_CONFIGS:-c2}; do
    timeout -k 10 120 python -u tools/wave_trace.py $c > "$OUT/wave_trace_$c.json" 2> "$OUT/wave_trace_$c.err"
    rc=$?
    [ $rc -eq 0 ] || { cp /tmp/librt_amd.base.so "$LIB"; echo "wave trace $c rc=$rc"; tail -20 "$OUT/wave_trace_$c.err"; exit 20; }
    python3 -c "import json; d=json.load(open('$OUT/wave_trace_$c.json')); print('$c', d['span_us'], d.get('attribution_us'), d.get('mean_phase_us'), d.get('resident_max'))"
  done
  cp /tmp/librt_amd.base.so "$LIB"
fi
if want c4n1; then
  timeout -k 10 180 python -u tools/c4_n1_probe.py > "$OUT/c4_n1.json" 2> "$OUT/c4_n1.err" \
      || { echo "c4_n1 probe failed"; tail -20 "$OUT/c4_n1.err"; exit 21; }
  cat "$OUT/c4_n1.json"
fi
if want hostw; then
  timeout -k 10 120 ./tools/_mb_hostwrite > "$OUT/hostwrite.jsonl" 2> "$OUT/hostwrite.err" \
      || { echo "hostwrite failed"; tail -20 "$OUT/hostwrite.err"; exit 23; }
  cat "$OUT/hostwrite.jsonl"
fi
if want refill; then
  for c in ${REFILL_CONFIGS:-c5 c2}; do
    gx=960; case "$c" in c2pair) gx=120;; c5pair) gx=480;; c2*) gx=240;; esac
    timeout -k 10 120 ./tools/_var/mb_refill $c $gx >> "$OUT/refill.jsonl" 2> "$OUT/refill.err" \
        || { echo "refill $c failed"; tail -20 "$OUT/refill.err"; exit 24; }
  done
  cat "$OUT/refill.jsonl"
fi
if want abenv; then
  timeout -k 10 ${AB_TIMEOUT:-600} python -u tools/ab_env.py ${CONFIGS:-c2,c3,c5} ${ROUNDS:-9} ${ABENV_MODES} \
      > "$OUT/abenv.jsonl" 2> "$OUT/abenv.err" || { echo "abenv failed"; tail -20 "$OUT/abenv.err"; exit 25; }
  cat "$OUT/abenv.jsonl"
fi
if want compsim; then
  timeout -k 10 180 python -u tools/compaction_sim.py ${COMPSIM_CONFIGS:-c2,c3,c5} > "$OUT/compaction_sim.jsonl" \
      2> "$OUT/compaction_sim.err" || { echo "compaction_sim failed"; tail -20 "$OUT/compaction_sim.err"; exit 26; }
  cat "$OUT/compaction_sim.jsonl"
fi
if want sdma; then
  timeout -k 10 120 ./tools/_var/mb_sdma > "$OUT/sdma.jsonl" 2> "$OUT/sdma.err" || { echo "sdma probe failed"; tail -20 "$OUT/sdma.err"; exit 27; }
  cat "$OUT/sdma.jsonl"
fi
if want copyab; then
  SETTINGS=${COPY_SETTINGS:-0:16,3:0,1:0} timeout -k 10 300 python -u tools/copy_ab.py > "$OUT/copy_ab.json" \
      2> "$OUT/copy_ab.err" || { echo "copy_ab failed"; tail -20 "$OUT/copy_ab.err"; exit 28; }
  cat "$OUT/copy_ab.json"
fi
if want ab; then
  VARS=${VARS:-} timeout -k 10 ${AB_TIMEOUT:-600} python -u tools/ab_libs.py ${CONFIGS:-c2,c3,c5} ${ROUNDS:-9} \
      > "$OUT/ab.jsonl" 2> "$OUT/ab.err" || { echo "ab failed"; tail -20 "$OUT/ab.err"; exit 22; }
  cat "$OUT/ab.jsonl"
fi
if want mbunpack; then
  timeout -k 10 60 ./tools/_mb_unpack > "$OUT/mb_unpack.jsonl" 2>&1 || { echo "mb_unpack failed"; tail -5 "$OUT/mb_unpack.jsonl"; exit 31; }
  cat "$OUT/mb_unpack.jsonl"
fi
if want queues; then
  PARTS=5 timeout -k 10 150 python -u tools/c4_gap_probe.py > "$OUT/queues.jsonl" 2> "$OUT/queues.err" \
      || { echo "queues failed"; tail -5 "$OUT/queues.err"; exit 32; }
  cat "$OUT/queues.jsonl"
  (cd /tmp && export TMPDIR=/tmp && PARTS=5 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
      -d "$OUT/queues_trace" -o run -- python3 "$ROOT/tools/c4_gap_probe.py" > "$OUT/queues_trace.log" 2>&1) \
      || { echo "queues trace failed"; tail -5 "$OUT/queues_trace.log"; exit 33; }
  python3 tools/queue_map.py "$OUT/queues_trace"
fi
if want c4probe; then
  timeout -k 10 500 python -u tools/c4_gap_probe.py > "$OUT/c4probe.jsonl" 2> "$OUT/c4probe.err" \
      || { echo "c4probe failed"; tail -5 "$OUT/c4probe.err"; exit 34; }
  cat "$OUT/c4probe.jsonl"
fi
if want count; then
  timeout -k 10 400 bash tools/count.sh || { echo "count failed"; exit 35; }
fi
if want profsdma; then
  timeout -k 10 300 bash tools/prof_sdma.sh || { echo "prof_sdma failed"; exit 36; }
fi
if want bench; then
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
      || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 3; }
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms_serial'], r['interval_ms_in_flight'], {k: v.get('kernel_ms_serial') for k, v in d.get('configs', {}).items()}, json.dumps(d.get('c4', {}))[:1200], json.dumps(d.get('drop_in', {}))[:900])"
fi
if want rehearse; then
  timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline \
      > "$OUT/rehearse.json" 2> "$OUT/rehearse.err" || { echo "rehearsal failed"; tail -30 "$OUT/rehearse.err"; exit 4; }
  python3 -c "import json; d=json.load(open('$OUT/rehearse.json')); print(d['n_gpus'], d['value'], d['config']['parallelism']); print(json.dumps(d.get('c4'))[:1500])"
fi
if want prof; then
  cd /tmp && export TMPDIR=/tmp
  for c in ${CONFIGS:-c2 c3 c5}; do
    steps=100; [ "$c" = "c5" ] && steps=30
    rm -rf "$OUT/prof1_$c"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof1_$c" -o run -- \
        python3 "$ROOT/bench.py" --config $c --steps $steps --warmup 5 --no-cpu-baseline --profile-kernel-only \
        --frames-in-flight 1 > "$OUT/prof1_bench_$c.json" 2> "$OUT/prof1_$c.err" \
        || { echo "rocprof $c failed"; tail -20 "$OUT/prof1_$c.err"; exit 5; }
    echo "== $c"; find "$OUT/prof1_$c" -name "*kernel_stats.csv" -exec head -3 {} \;
  done
  cd "$ROOT"
fi
if want pmc; then
  for c in ${CONFIGS:-c2 c3 c5}; do
    CONFIG=$c timeout -k 10 900 bash tools/pmc.sh > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed"; tail -20 "$OUT/pmc_$c.log"; exit 6; }
    tail -2 "$OUT/pmc_$c.log"
  done
fi
