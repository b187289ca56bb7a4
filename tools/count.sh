#!/bin/bash
# Exact per-variant instruction counts of rt_render_kernel (tools/count.py), one rocprofv3 --pmc run each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/count
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-full d0 nospheres noboard empty nolights}; do
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-trace \
     --output-format csv -d "$OUT/$v" -o run -- python3 "$ROOT/tools/count.py" $v ${CONFIG:-c2} > "$OUT/$v.log" 2>&1 || { echo "variant $v failed"; tail -3 "$OUT/$v.log"; exit 5; }
  python3 "$ROOT/tools/pmc_summary.py" "$OUT/$v" | python3 -c "
import json,sys; d=json.load(sys.stdin)
for k,c in d.items():
    if k.startswith('rt_render'):
        print('$v', {x: round(y/1e3) for x, y in c.items() if x.startswith('SQ')}, 'k-instr')"
done
