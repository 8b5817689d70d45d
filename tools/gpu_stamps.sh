# Phase stamps of the warp pipeline kernel (profiling build) + quick parity + warp-only bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 150 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 60 --timeout-method thread -k "(test_fused_nhwc_kernels and pipeline) or repeat" > $O/quick.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/quick.log; [ $rc -ne 0 ] && exit $rc
for w in 2 3; do
timeout -k 10 120 python -u tools/warp_stamps.py --wgs $w > $O/stamps$w.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 --warp-wgs $w > $O/bench_pc$w.log 2>&1 || exit $?
done
exit 0
