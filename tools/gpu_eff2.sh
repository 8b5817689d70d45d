set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/eff2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_effnet.py tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --backbone efficientnet_b3 --steps 20 --warmup 3 --cpu-iters 0 > $O/bench_b3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/warp.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 bench.py --backbone efficientnet_b3 --steps 5 --warmup 2 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
exit 0
