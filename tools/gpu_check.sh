#!/bin/bash
# One GPU-box session: parity tests, a bench line, a rocprofv3 kernel-trace summary.
# Stops at the first crash / timeout (exit >1 from pytest, any failure afterwards).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
rocm-smi --showproductname > "$OUT/smi.txt" 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -15 "$OUT/gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 3; }
cat "$OUT/bench.json"
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  # the kernel-only bench (no parity render): its 100 timed dispatches dominate the stats; the first
  # dispatch of the view is the tile-order calibration render (rt_order_kernel follows it once)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --steps 100 --warmup 5 --no-cpu-baseline --profile-kernel-only > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
      || { echo "rocprof failed"; tail -20 "$OUT/prof.err"; exit 4; }
  find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \;
  cd "$ROOT" && python3 tools/kernel_gaps.py "$OUT/prof" | tee "$OUT/prof_dispatches.json"
fi
exit $rc
