# Round 5 pass q: counters of the fp16-operand conv kernels (tools/conv_h16_micro.py shapes), one PMC group per run.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
S=${SHAPES:-head2_fwd,l1_c3,l2_c2,l1_c1}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
P3="SQ_WAVES TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P4="SQ_WAVES WRITE_SIZE"
P5="SQ_WAVES FETCH_SIZE"
n=1
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$n -o run -- python3 tools/conv_h16_micro.py --only $S --reps 2 ${WGRAD:---wgrad} > $O/p$n.log 2>&1 || exit $?
  n=$((n+1))
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/conv_h16_micro.py --only $S --reps 3 ${WGRAD:---wgrad} > $O/kt.log 2>&1 || exit $?
exit 0
