# Per-layer SQ counters of the conv kernel (MFMA busy, wait/issue stalls, clock) for a few layer shapes.
# EXTRA="--arith bf16x6" selects the split-bf16 kernels.
# usage (on the box): bash tools/gpu_conv_pmc.sh <tag> <layer>...
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for L in "$@"; do
  timeout -k 10 120 python -u tools/conv_micro.py $L ${EXTRA:-} --iters 5 --rounds 1 > $O/time_$L.txt 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/p1_$L -o run -- python3 tools/conv_micro.py $L ${EXTRA:-} --iters 3 --rounds 1 > $O/p1_$L.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $O/p2_$L -o run -- python3 tools/conv_micro.py $L ${EXTRA:-} --iters 3 --rounds 1 > $O/p2_$L.log 2>&1 || exit $?
done
exit 0
