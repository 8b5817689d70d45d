# PMC passes on the fused warp (warp-only bench), default build and skeleton ablation (BEV_WARP_DEBUG=15).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wpmc; mkdir -p $O
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_WAIT_INST_SCA" \
           "SQ_BARRIER_CYCLES SQ_WAIT_BARRIER" "SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_SENDMSG" "TA_BUSY_avr TD_BUSY_avr TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  for d in 0 15; do
    BEV_WARP_DEBUG=$d timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d $O/p${i}_d$d -o run -- python3 $R/bench.py --warp-only --steps 3 --warmup 1 --cpu-iters 0 > $O/p${i}_d$d.log 2>&1
    echo "pass $i dbg $d rc=$?" >> $O/status.log
  done
done
exit 0
