#!/bin/bash
# One GPU-box session (round 3): the GPU tests, the default bench line, then (PROFILE=1) one-stream rocprofv3
# kernel-trace summaries of the kernel-only bench at c2, c3 and c5 (AverageNs = the launch duration: the
# roofline's denominator).  Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} \
      > "$OUT/gpu_tests.log" 2>&1
  rc=$?
  tail -15 "$OUT/gpu_tests.log"
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" \
      || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 3; }
  cat "$OUT/bench.json"
fi
[ "${PROFILE:-0}" = "1" ] || exit 0
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-c2 c3 c5}; do
  steps=100; [ "$c" = "c5" ] && steps=30
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof1_$c" -o run -- \
      python3 "$ROOT/bench.py" --config $c --steps $steps --warmup 5 --no-cpu-baseline --profile-kernel-only \
      --frames-in-flight 1 > "$OUT/prof1_bench_$c.json" 2> "$OUT/prof1_$c.err" \
      || { echo "rocprof $c failed"; tail -20 "$OUT/prof1_$c.err"; exit 4; }
  echo "== $c"; find "$OUT/prof1_$c" -name "*kernel_stats.csv" -exec head -3 {} \;
done
