# Warp study: ablation timings (BEV_WARP_DEBUG bits) + PMC passes on the default fused warp.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wstudy; mkdir -p $O
for d in 0 1 2 4 8 6 10 12 14 15; do
  BEV_WARP_DEBUG=$d timeout -k 10 120 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/dbg$d.log 2>&1 || exit $?
done
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR" \
           "SQ_BARRIER_CYCLES SQ_WAIT_BARRIER" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d $O/p$i -o run -- python3 $R/bench.py --warp-only --steps 3 --warmup 1 --cpu-iters 0 > $O/p$i.log 2>&1 || exit $?
done
exit 0
