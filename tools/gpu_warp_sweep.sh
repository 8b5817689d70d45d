set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider > gpurun_out/warp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/warp_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for kb in 40 60 76; do
  BEV_WARP_LDS_KB=$kb timeout -k 10 300 python bench.py --warp-only --steps 30 --warmup 5 --cpu-iters 0 > gpurun_out/warp_kb$kb.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-iters 0 > gpurun_out/bench2.log 2>&1
