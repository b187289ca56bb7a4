#!/bin/bash
# Round-4 profile session: GPU tests, the default bench line, one-stream rocprofv3 kernel-trace summaries of the
# kernel-only bench at c2 / c3 / c5 (AverageNs = the launch duration, the roofline's denominator) and the PMC
# passes (tools/pmc.sh) per config.  STEPS selects parts; each GPU step has its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
want() { case " ${STEPS:-tests bench prof pmc} " in *" $1 "*) return 0;; esac; return 1; }
if want tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
if want bench; then
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
      || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 3; }
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_serial'], d['roofline']['interval_ms_in_flight'], {k: v.get('kernel_ms_serial') for k, v in d.get('configs', {}).items()}, json.dumps(d.get('drop_in', {}))[:900], d['cpu_baseline']['kind'], d['cpu_baseline']['value'])"
fi
if want prof; then
  cd /tmp && export TMPDIR=/tmp
  for c in ${CONFIGS:-c2 c3 c5}; do
    steps=100; [ "$c" = "c5" ] && steps=30
    rm -rf "$OUT/prof1_$c"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof1_$c" -o run -- \
        python3 "$ROOT/bench.py" --config $c --steps $steps --warmup 5 --no-cpu-baseline --profile-kernel-only \
        --frames-in-flight 1 > "$OUT/prof1_bench_$c.json" 2> "$OUT/prof1_$c.err" \
        || { echo "rocprof $c failed"; tail -20 "$OUT/prof1_$c.err"; exit 4; }
    echo "== $c"; find "$OUT/prof1_$c" -name "*kernel_stats.csv" -exec head -3 {} \;
  done
  cd "$ROOT"
fi
if want pmc; then
  for c in ${CONFIGS:-c2 c3 c5}; do
    CONFIG=$c timeout -k 10 900 bash tools/pmc.sh > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed"; tail -20 "$OUT/pmc_$c.log"; exit 5; }
    tail -2 "$OUT/pmc_$c.log"
  done
fi
