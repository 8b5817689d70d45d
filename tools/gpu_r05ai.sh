# Round 5 pass ai: the ordered kernel trace of one AMP BEVNet training step (which launch is which layer)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/ttrace -o run -- python3 tools/train_step_bench.py --steps 1 --warmup 1 --bevnet --amp > $O/ttrace.log 2>&1 || exit $?
exit 0
