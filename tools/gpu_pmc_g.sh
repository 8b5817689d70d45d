# PMC HBM-traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs) over the bench command.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcg; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-iters 0 > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-iters 0 > $O/pmc_write.log 2>&1 || exit $?
exit 0
