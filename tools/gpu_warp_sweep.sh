set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider > gpurun_out/warp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/warp_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
BEV_WARP_POOL_KB=8 timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider -k "full_size or fused" > gpurun_out/warp_tests_pool8.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/warp_tests_pool8.log
if [ $rc -ne 0 ]; then exit $rc; fi
for kb in 48 72 100; do
  BEV_WARP_POOL_KB=$kb timeout -k 10 300 python bench.py --warp-only --steps 30 --warmup 5 --cpu-iters 0 > gpurun_out/warp_pool$kb.log 2>&1 || exit $?
done
BEV_WARP_NO_DMA=1 timeout -k 10 300 python bench.py --warp-only --steps 30 --warmup 5 --cpu-iters 0 > gpurun_out/warp_nodma.log 2>&1 || exit $?
