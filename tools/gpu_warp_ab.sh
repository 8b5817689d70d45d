# Fused-warp GPU pass: warp parity tests, then warp-only bench of both fused kernels + rocprof stats.
# usage (on the box): bash tools/gpu_warp_ab.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/warp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/warp_tests.log; [ $rc -ne 0 ] && exit $rc
for k in dma register; do
  timeout -k 10 300 python -u bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 --warp-kernel $k > $O/bench_$k.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --warp-only --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
exit 0
