#!/bin/bash
# Round-4 session B: GPU tests at HEAD, the wave-slot probe (SGPR thresholds at 63 VGPRs), the in-process A/B of
# tools/_var builds (VARS) at c2/c3/c5, and the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
want() { case " ${STEPS:-tests ab bench copy2} " in *" $1 "*) return 0;; esac; return 1; }
if want tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} \
      > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -5 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
if want slots && [ -x tools/_var/mb_slots ]; then
  timeout -k 10 60 tools/_var/mb_slots > "$OUT/slots.jsonl" 2>&1 || { echo "slots failed"; cat "$OUT/slots.jsonl"; exit 5; }
  cat "$OUT/slots.jsonl"
fi
if want ab; then
  VARS=${VARS:-old,sg96,sg80} timeout -k 10 600 python -u tools/ab_libs.py ${CONFIGS:-c2,c3,c5} ${ROUNDS:-9} \
      > "$OUT/ab.jsonl" 2> "$OUT/ab.err" || { echo "ab failed"; tail -20 "$OUT/ab.err"; exit 6; }
  cat "$OUT/ab.jsonl"
fi
if want bench; then
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
      || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 3; }
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_serial'], d['roofline']['interval_ms_in_flight'], {k: v.get('kernel_ms_serial') for k, v in d.get('configs', {}).items()}, d.get('drop_in', {}).get('moving_camera', {}).get('ms_per_frame'))"
fi
if want ctrace; then
  cd /tmp && export TMPDIR=/tmp
  for spec in ${CTRACE_SPECS:-"1 0 1" "0 16 2" "0 0 2"}; do
    set -- $(echo $spec | tr ',' ' ')
    rm -rf "$OUT/ctrace_$1_$2_$3"
    RT_COPY_KERNEL=${4:--1} RT_COPY_MODE=$1 RT_COPY_BLOCKS=$2 DEPTH=$3 timeout -k 10 120 rocprofv3 --kernel-trace \
        --memory-copy-trace --output-format csv \
        -d "$OUT/ctrace_$1_$2_$3" -o run -- python3 "$GRAFT_REPO_ROOT/tools/copy_trace.py" > "$OUT/ctrace_$1_$2_$3.json" \
        2> "$OUT/ctrace_$1_$2_$3.err" || { echo "ctrace $spec failed"; tail -5 "$OUT/ctrace_$1_$2_$3.err"; exit 7; }
    cat "$OUT/ctrace_$1_$2_$3.json"; python3 "$GRAFT_REPO_ROOT/tools/copy_trace.py" parse "$OUT/ctrace_$1_$2_$3"
  done
  cd "$GRAFT_REPO_ROOT"
fi
if want copy2; then
  for env in "RT_HOST_NONCOHERENT=0" "RT_HOST_NONCOHERENT=1" "RT_COPY_KERNEL=0"; do
    env $env SETTINGS=1:0,0:16,0:0 ROUNDS=3 timeout -k 10 200 python -u tools/copy_ab.py > "$OUT/copy2_$env.json" \
        2> "$OUT/copy2_$env.err" || { echo "copy2 $env failed"; tail -5 "$OUT/copy2_$env.err"; exit 8; }
    echo "$env"; python3 -c "import json; print(json.load(open('$OUT/copy2_$env.json'))['us_per_frame_median'])"
  done
fi
if want over; then
  timeout -k 10 120 python -u tools/overhead_probe.py > "$OUT/overhead.json" 2> "$OUT/overhead.err" \
      || { echo "overhead probe failed"; tail -20 "$OUT/overhead.err"; exit 13; }
  cat "$OUT/overhead.json"
fi
if want screen; then
  for n in 0 1 2; do
    RT_SCREEN_NEXT=$n RT_SCREEN_PROFILE=1 timeout -k 10 200 python -u tools/screen_bench.py demo 500 500 c2 640 360 \
        > "$OUT/screen_$n.json" 2> "$OUT/screen_$n.err" || { echo "screen $n failed"; tail -5 "$OUT/screen_$n.err"; exit 9; }
    echo "RT_SCREEN_NEXT=$n"; cat "$OUT/screen_$n.json"; grep rt_render_screen "$OUT/screen_$n.err" | tail -2
  done
fi
