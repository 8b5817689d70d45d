# Round 5 pass ap: the fused warp's channels-last output (bev_ipm_warp_fuse_nhwc_f32, forward_fused's inference
# default): warp / dist / C-ABI / smoke tests, then the default bench alternating with --warp-nchw, and the kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_warp_gpu.py tests/test_capi.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --cpu-iters 0 > $O/bench_cl_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --cpu-iters 0 --warp-nchw > $O/bench_nchw_$r.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
exit 0
