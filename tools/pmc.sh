#!/bin/bash
# PMC passes for the dominant kernel (one counter group per rocprofv3 run, --kernel-trace only beside
# --pmc, as MI355X_MICROARCH.md / the pool rules require).  Usage: CONFIG=c2 bash tools/pmc.sh
# PMC_GROUPS='A B;C D' overrides the counter groups (';' separates passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_${CONFIG:-c2}
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $group --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
     python3 "$ROOT/bench.py" --config ${CONFIG:-c2} --steps 10 --warmup 2 --profile-kernel-only --frames-in-flight 1 \
     > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($group) failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 5; }
  echo "pass $i ok: $group"
done < <(if [ -n "${PMC_GROUPS:-}" ]; then echo "$PMC_GROUPS" | tr ';' '\n'; else cat <<'GROUPS'
WRITE_SIZE
FETCH_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32
VALUUtilization VALUBusy
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR
GROUPS
fi)
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
