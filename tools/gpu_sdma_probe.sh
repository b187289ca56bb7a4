#!/bin/bash
# Which engine runs rt_render_packed_async's device-to-host copy, per runtime setting: timing (3 fresh processes
# each) and one kernel + memory-copy trace.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
for s in "NONE=1" "GPU_FORCE_BLIT_COPY_SIZE=0" "ROC_ENABLE_LARGE_BAR=0" "HSA_ENABLE_SDMA=1" "GPU_BLIT_ENGINE_TYPE=2"; do
  for r in 1 2 3; do
    env $s K=100 timeout -k 10 60 python3 tools/copy_trace.py > "$OUT/sdma_$s.$r.json" 2> "$OUT/sdma_$s.$r.err" \
        || { echo "$s failed"; tail -5 "$OUT/sdma_$s.$r.err"; exit 3; }
    echo "$s $(cat "$OUT/sdma_$s.$r.json")"
  done
  ( cd /tmp && export TMPDIR=/tmp && rm -rf "$OUT/sdmat_$s" && env $s K=40 timeout -k 10 90 rocprofv3 --kernel-trace \
      --memory-copy-trace --output-format csv -d "$OUT/sdmat_$s" -o run -- python3 "$ROOT/tools/copy_trace.py" \
      > /dev/null 2> "$OUT/sdmat_$s.err" ) || { echo "trace $s failed"; tail -5 "$OUT/sdmat_$s.err"; exit 4; }
  python3 - "$OUT/sdmat_$s" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
k = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
m = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
c = collections.Counter(r["Kernel_Name"][:40] for r in csv.DictReader(open(k[0]))) if k else {}
n = sum(1 for _ in csv.DictReader(open(m[0]))) if m else 0
print("   kernels:", dict(c), " memory copies:", n)
PY
done
