set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_backbone_gpu.py -q -x -p no:cacheprovider > gpurun_out/conv_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/conv_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_conv -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-iters 0 > gpurun_out/conv_prof_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-iters 0 > gpurun_out/conv_bench.log 2>&1
