# Conv change check: backbone/EfficientNet/head GPU tests, per-layer timings, default bench line.
# usage (on the box): bash tools/gpu_conv_ab.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/conv_micro.py --iters 10 --rounds 1 > $O/layers.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
exit 0
