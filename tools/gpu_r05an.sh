# Round 5 pass an: ordered kernel trace of the default bench (which launches / copies / idle gaps a step holds)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/btrace -o run -- python3 bench.py --steps 4 --warmup 2 --cpu-iters 0 > $O/btrace.log 2>&1 || exit $?
exit 0
