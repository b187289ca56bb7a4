#!/bin/bash
# Diagnostic GPU session: wave-level event counters (RT_COUNTERS variant) and an in-process A/B of variant builds
# (tools/_var/*, VARS=comma list) against the in-tree library.  CONFIGS / ROUNDS select the A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
if [ -f tools/_var/cnt/librt_amd.so ] && [ "${COUNTERS:-1}" = "1" ]; then
  timeout -k 10 200 python -u tools/counters.py ${CNT_CONFIGS:-c2,c3,c5} > "$OUT/counters.jsonl" 2> "$OUT/counters.err" \
      || { echo "counters failed"; tail -20 "$OUT/counters.err"; exit 2; }
  cat "$OUT/counters.jsonl"
fi
VARS=${VARS:-cheap,lazy0} timeout -k 10 500 python -u tools/ab_libs.py ${CONFIGS:-c2,c3,c5} ${ROUNDS:-9} > "$OUT/ab.jsonl" 2> "$OUT/ab.err" \
    || { echo "ab failed"; tail -20 "$OUT/ab.err"; exit 3; }
cat "$OUT/ab.jsonl"
