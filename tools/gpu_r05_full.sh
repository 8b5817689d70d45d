# Round-5 full GPU pass: every GPU test, the smoke, the default bench line, a rocprofv3 kernel-trace summary of the
# bench, and the camera-shard (K5) and EfficientNet-B3 (K4) lines.
# usage (on the box): bash tools/gpu_r05_full.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --camera-shard --steps 10 --warmup 2 --cpu-iters 0 > $O/cam.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --backbone efficientnet_b3 --steps 20 --warmup 3 --cpu-iters 0 > $O/effb3.log 2>&1 || exit $?
if [ -n "${TRAIN:-}" ]; then
  timeout -k 10 300 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_amp.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
fi
exit 0
