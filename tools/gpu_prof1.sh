set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rocprofv3 -L > gpurun_out/prof/counters_list.txt 2>&1 || true
# kernel trace of the full bench (backbone + warp)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/full -o run -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-iters 0 > gpurun_out/prof/full_bench.log 2>&1 || exit $?
# counters on the warp kernel (separate passes)
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/prof/pmc1 -o run -- python3 $R/bench.py --warp-only --steps 3 --warmup 1 --cpu-iters 0 > gpurun_out/prof/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/prof/pmc2 -o run -- python3 $R/bench.py --warp-only --steps 3 --warmup 1 --cpu-iters 0 > gpurun_out/prof/pmc2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/prof/pmc3 -o run -- python3 $R/bench.py --warp-only --steps 3 --warmup 1 --cpu-iters 0 > gpurun_out/prof/pmc3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/pmc4 -o run -- python3 $R/bench.py --warp-only --steps 3 --warmup 1 --cpu-iters 0 > gpurun_out/prof/pmc4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/pmc5 -o run -- python3 $R/bench.py --warp-only --steps 3 --warmup 1 --cpu-iters 0 > gpurun_out/prof/pmc5.log 2>&1 || exit $?
