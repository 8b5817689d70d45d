# Iteration run: backbone + warp parity, warp timing/ablation, conv layer micro, full bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/iter; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_backbone_gpu.py tests/test_warp_gpu.py -q -x -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
BEV_WARP_POOL_KB=8 timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider -k "full_size or fused" > $O/tests_pool8.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests_pool8.log; [ $rc -ne 0 ] && exit $rc
for d in 0 1 15; do
  BEV_WARP_DEBUG=$d timeout -k 10 300 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/warp_dbg$d.log 2>&1 || exit $?
done
timeout -k 10 600 python3 tools/conv_micro.py --iters 10 > $O/micro.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --cpu-iters 0 > $O/bench.log 2>&1 || exit $?
exit 0
