# Two SQ PMC passes + a kernel trace of an arbitrary python command (each its own rocprofv3 run).
# usage (on the box): bash tools/gpu_pmc_cmd.sh <tag> <python script> [args...]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
timeout -s KILL 170 rocprofv3 --pmc $P1 --output-format csv -d $O/p1 -o run -- python3 "$@" > $O/p1.log 2>&1 || exit $?
timeout -s KILL 170 rocprofv3 --pmc $P2 --output-format csv -d $O/p2 -o run -- python3 "$@" > $O/p2.log 2>&1 || exit $?
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 "$@" > $O/kt.log 2>&1 || exit $?
exit 0
