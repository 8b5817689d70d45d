set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/wab2; mkdir -p $O
BEV_WARP_TH=16 timeout -k 10 600 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 -k "fused" > $O/tests16.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests16.log; [ $rc -ne 0 ] && exit $rc
b() { n=$1; shift; timeout -k 10 120 env "$@" python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/$n.log 2>&1; }
b th8 BEV_WARP_TH=8 || exit $?
b th16 BEV_WARP_TH=16 || exit $?
b th32 BEV_WARP_TH=32 || exit $?
b th16_p100 BEV_WARP_TH=16 BEV_WARP_POOL_KB=100 || exit $?
b th16_dbg15 BEV_WARP_TH=16 BEV_WARP_DEBUG=15 || exit $?
b th16_dbg2 BEV_WARP_TH=16 BEV_WARP_DEBUG=2 || exit $?
b th16_dbg4 BEV_WARP_TH=16 BEV_WARP_DEBUG=4 || exit $?
BEV_WARP_TH=16 BEV_WARP_DEBUG=64 timeout -k 10 120 python tools/warp_phases_v2.py > $O/ph16.log 2>&1 || exit $?
exit 0
