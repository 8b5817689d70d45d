# Warp parity tests + warp-only timing (default, OCC 2) + kernel trace of the default.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/warp; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/bench_default.log 2>&1 || exit $?
BEV_WARP_OCC=2 timeout -k 10 300 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/bench_occ2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --warp-only --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
exit 0
