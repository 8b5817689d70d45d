set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/occ3; mkdir -p $O
BEV_WARP_OCC=3 timeout -k 10 600 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 -k fused > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
b() { n=$1; shift; timeout -k 10 120 env "$@" python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/$n.log 2>&1; }
b occ4 BEV_WARP_OCC=4 || exit $?
b occ3 BEV_WARP_OCC=3 || exit $?
b occ3_p52 BEV_WARP_OCC=3 BEV_WARP_POOL_KB=51 || exit $?
b occ3_p44 BEV_WARP_OCC=3 BEV_WARP_POOL_KB=44 || exit $?
b occ4_p38 BEV_WARP_OCC=4 BEV_WARP_POOL_KB=37 || exit $?
b occ3_dbg1 BEV_WARP_OCC=3 BEV_WARP_DEBUG=1 || exit $?
b occ4_dbg1 BEV_WARP_OCC=4 BEV_WARP_DEBUG=1 || exit $?
exit 0
