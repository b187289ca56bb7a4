#!/bin/bash
# One GPU-box session (round 4): GPU tests, the bench guard (launch decisions, watchdog rc), the draw() copy A/B
# and the COPY-transport gather A/B.  STEPS selects parts (default all).  Each GPU step has its own limit; the
# script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
want() { case " ${STEPS:-tests guard copy c4 over diag bench} " in *" $1 "*) return 0;; esac; return 1; }
if want tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} \
      > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -5 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
if want guard; then
  timeout -k 10 900 bash tools/gpu_bench_guard.sh > "$OUT/guard.log" 2>&1
  rc=$?; cat "$OUT/guard.log"; [ $rc -eq 0 ] || { echo "guard rc=$rc"; exit 10; }
fi
if want copy; then
  timeout -k 10 300 python -u tools/copy_ab.py > "$OUT/copy_ab.json" 2> "$OUT/copy_ab.err" \
      || { echo "copy_ab failed"; tail -20 "$OUT/copy_ab.err"; exit 11; }
  cat "$OUT/copy_ab.json"
fi
if want c4; then
  timeout -k 10 300 python -u tools/c4_copy_probe.py > "$OUT/c4_copy.json" 2> "$OUT/c4_copy.err" \
      || { echo "c4 probe failed"; tail -20 "$OUT/c4_copy.err"; exit 12; }
  cat "$OUT/c4_copy.json"
fi
if want over; then
  timeout -k 10 120 python -u tools/overhead_probe.py > "$OUT/overhead.json" 2> "$OUT/overhead.err" \
      || { echo "overhead probe failed"; tail -20 "$OUT/overhead.err"; exit 13; }
  cat "$OUT/overhead.json"
fi
if want diag; then
  timeout -k 10 700 bash tools/gpu_diag.sh > "$OUT/diag.log" 2>&1
  rc=$?; cat "$OUT/diag.log"; [ $rc -eq 0 ] || { echo "diag rc=$rc"; exit 14; }
fi
if want bench; then
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
      || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 3; }
  cat "$OUT/bench.json"
fi
