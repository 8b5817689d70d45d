# Full GPU pass: parity tests, smoke, layer micro-bench, bench, rocprof kernel trace of the bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/round
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/round/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/round/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/conv_micro.py --iters 10 > gpurun_out/round/conv_micro.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/round/bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/round/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-iters 0 > gpurun_out/round/prof_bench.log 2>&1 || exit $?
