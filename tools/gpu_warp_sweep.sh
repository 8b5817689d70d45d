set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider > gpurun_out/warp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/warp_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "BEV_WARP_RING_KB=3" "BEV_WARP_BLOCK_DMA=1"; do
env $cfg timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider -k "full_size or fused" > gpurun_out/warp_tests_$cfg.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/warp_tests_$cfg.log; [ $rc -ne 0 ] && exit $rc
done
for kb in 10 13 20; do
  BEV_WARP_RING_KB=$kb timeout -k 10 300 python bench.py --warp-only --steps 30 --warmup 5 --cpu-iters 0 > gpurun_out/warp_ring$kb.log 2>&1 || exit $?
done
exit 0
