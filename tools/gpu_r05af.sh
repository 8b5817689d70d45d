# Round 5 pass af: HBM traffic of the default bench workload after the stem + max-pool fusion -- the two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs), reduced afterwards by tools/pmc_traffic.py.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-iters 0 > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-iters 0 > $O/write.log 2>&1 || exit $?
exit 0
