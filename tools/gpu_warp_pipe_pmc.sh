# SQ / LDS / clock counters of the fused warp in the full bench pipeline AND in warp-only mode (PMC passes of
# their own), the LDS exec-mask microbenchmark, and a kernel trace of the bench.
# usage (on the box): bash tools/gpu_warp_pipe_pmc.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
if [ -x tools/lds_exec_micro ]; then timeout -k 10 60 ./tools/lds_exec_micro > $O/lds_exec_micro.txt 2>&1 || exit $?; fi
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
for mode in pipe warp; do
  X=""; [ $mode = warp ] && X="--warp-only"
  timeout -s KILL 170 rocprofv3 --pmc $P1 --output-format csv -d $O/${mode}_p1 -o run -- python3 bench.py $X --steps 6 --warmup 2 --cpu-iters 0 > $O/${mode}_p1.log 2>&1 || exit $?
  timeout -s KILL 170 rocprofv3 --pmc $P2 --output-format csv -d $O/${mode}_p2 -o run -- python3 bench.py $X --steps 6 --warmup 2 --cpu-iters 0 > $O/${mode}_p2.log 2>&1 || exit $?
  timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${mode}_kt -o run -- python3 bench.py $X --steps 10 --warmup 2 --cpu-iters 0 > $O/${mode}_kt.log 2>&1 || exit $?
done
exit 0
