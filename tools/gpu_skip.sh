set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/skip; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
b() { n=$1; shift; timeout -k 10 120 env "$@" python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/$n.log 2>&1; }
b occ4 BEV_WARP_OCC=4 || exit $?
b occ2 BEV_WARP_OCC=2 || exit $?
b occ4_dbg15 BEV_WARP_OCC=4 BEV_WARP_DEBUG=15 || exit $?
exit 0
