# PMC passes on the fused warp (warp-only bench): default kernel and the legacy v2 kernel.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc3; mkdir -p $O
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  for v in 0 1; do
    if [ $v = 1 ]; then export BEV_WARP_V2=1; else unset BEV_WARP_V2; fi
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d $O/p${i}_v$v -o run -- python3 $R/bench.py --warp-only --steps 3 --warmup 1 --cpu-iters 0 > $O/p${i}_v$v.log 2>&1
    echo "pass $i v$v rc=$?" >> $O/status.log
  done
done
exit 0
