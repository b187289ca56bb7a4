#!/bin/bash
# Exact per-variant instruction counts of rt_render_kernel (tools/count.py), one rocprofv3 --pmc run each.
# VARIANTS: scene variants (tools/count.py); LIBS: "base" (the in-tree library) and/or tools/_ab/<name> builds
# (tools/ablate.sh: ablate1 = the prologue alone, ablate2 = trace without stores), each run with RT_LIB_PATH.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/count
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for lib in ${LIBS:-base}; do
  if [ "$lib" = base ]; then unset RT_LIB_PATH; tag=""; else export RT_LIB_PATH=$ROOT/tools/_ab/$lib/librt_amd.so; tag="${lib}_"; fi
  for v in ${VARIANTS:-full d0 nospheres noboard empty nolights}; do
    timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-trace \
       --output-format csv -d "$OUT/$tag$v" -o run -- python3 "$ROOT/tools/count.py" $v ${CONFIG:-c2} > "$OUT/$tag$v.log" 2>&1 || { echo "variant $tag$v failed"; tail -3 "$OUT/$tag$v.log"; exit 5; }
    python3 "$ROOT/tools/pmc_summary.py" "$OUT/$tag$v" > "$OUT/$tag$v.json"
    python3 -c "
import json; d=json.load(open('$OUT/$tag$v.json'))
for k,c in d.items():
    if 'rt_render' in k and c.get('_dispatches', 0) > 1:
        w = c['SQ_WAVES']; print('$tag$v', k[:48], {x[8:]: round(y / w, 1) for x, y in c.items() if x.startswith('SQ_INSTS')}, 'per wave')"
  done
done
unset RT_LIB_PATH
