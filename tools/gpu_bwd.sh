# Warp backward (LDS-reduced scatter) parity + training-step timing and kernel profile.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/bwd; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train.py -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/train_step_bench.py --steps 5 > $O/hot.log 2>&1 || exit $?
timeout -k 10 300 python tools/train_step_bench.py --steps 3 --bevnet > $O/bevnet.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/train_step_bench.py --steps 2 --warmup 1 > $O/prof.log 2>&1 || exit $?
exit 0
