# Round 5 pass as: the channels-last fused-warp store with the streaming (nt) policy: bench alternating with --warp-nchw,
# and the eager-loss training step (graphed loss removed) x2.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --cpu-iters 0 > $O/bench_cl_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --cpu-iters 0 --warp-nchw > $O/bench_nchw_$r.log 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 8 --bevnet --amp > $O/train_$r.log 2>&1 || exit $?
done
exit 0
