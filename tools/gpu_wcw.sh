set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/wcw; mkdir -p $O
BEV_WARP_CW=32 timeout -k 10 600 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 -k "fused" > $O/tests32.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests32.log; [ $rc -ne 0 ] && exit $rc
b() { n=$1; shift; timeout -k 10 120 env "$@" python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/$n.log 2>&1; }
b cw64 BEV_WARP_CW=64 || exit $?
b cw32 BEV_WARP_CW=32 || exit $?
b cw32_p30 BEV_WARP_CW=32 BEV_WARP_POOL_KB=30 || exit $?
b cw32_dbg15 BEV_WARP_CW=32 BEV_WARP_DEBUG=15 || exit $?
b cw32_dbg2 BEV_WARP_CW=32 BEV_WARP_DEBUG=2 || exit $?
b cw32_dbg1 BEV_WARP_CW=32 BEV_WARP_DEBUG=1 || exit $?
BEV_WARP_CW=32 BEV_WARP_DEBUG=64 timeout -k 10 120 python tools/warp_phases_v2.py > $O/ph32.log 2>&1 || exit $?
exit 0
