#!/bin/bash
# One GPU-box session: the default bench line, then rocprofv3 kernel-trace summaries of the kernel-only bench
# at c2, c3 and c5 (each step under its own time limit; stop at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 3; }
cat "$OUT/bench.json"
[ "${PROFILE:-1}" = "1" ] || exit 0
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-c2 c3 c5}; do
  steps=100; [ "$c" = "c5" ] && steps=30
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o run -- \
      python3 "$ROOT/bench.py" --config $c --steps $steps --warmup 5 --no-cpu-baseline --profile-kernel-only \
      > "$OUT/prof_bench_$c.json" 2> "$OUT/prof_$c.err" || { echo "rocprof $c failed"; tail -20 "$OUT/prof_$c.err"; exit 4; }
  echo "== $c"; find "$OUT/prof_$c" -name "*kernel_stats.csv" -exec head -3 {} \;
  (cd "$ROOT" && python3 tools/kernel_gaps.py "$OUT/prof_$c" $steps | tee "$OUT/prof_dispatches_$c.json")
done
