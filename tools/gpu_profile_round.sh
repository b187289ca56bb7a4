set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_bench_prof.sh > gpurun_out/prof_all.log 2>&1 || { echo "bench/prof failed"; tail -20 gpurun_out/prof_all.log; exit 3; }
G="WRITE_SIZE;FETCH_SIZE;SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;VALUUtilization VALUBusy"
for c in c2 c3 c5; do
  CONFIG=$c PMC_GROUPS="$G" bash tools/pmc.sh > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -20 gpurun_out/pmc_$c.log; exit 4; }
  echo "pmc $c ok"
done
