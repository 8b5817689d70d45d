set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_backbone_gpu.py -q -x -p no:cacheprovider > gpurun_out/conv_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/conv_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 tools/conv_micro.py --iters 10 --tiles 1 2 3 > gpurun_out/conv_ab.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-iters 0 > gpurun_out/conv_bench.log 2>&1
