# Warp parity (default + small pool) and v1/v2 timing A/B.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/wab; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
BEV_WARP_POOL_KB=8 timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider -k "full_size or fused" > $O/tests_pool8.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests_pool8.log; [ $rc -ne 0 ] && exit $rc
for cfg in "X=1" "BEV_WARP_V1=1" "BEV_WARP_OCC=2" "BEV_WARP_POOL_KB=48" "BEV_WARP_POOL_KB=28"; do
  env $cfg timeout -k 10 300 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/bench_$cfg.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --warp-only --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
exit 0
