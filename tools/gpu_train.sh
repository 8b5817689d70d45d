# Training-step timing (BASELINE config 3 shape) + rocprof kernel summary of the BEVNet step.
# usage (on the box): bash tools/gpu_train.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u tools/train_step_bench.py --steps 5 > $O/hot.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/train_step_bench.py --steps 5 --bevnet > $O/bevnet.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet > $O/prof.log 2>&1 || exit $?
exit 0
