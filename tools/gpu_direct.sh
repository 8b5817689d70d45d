set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/direct; mkdir -p $O
BEV_WARP_DIRECT=1 timeout -k 10 600 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 -k fused > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
b() { n=$1; shift; timeout -k 10 120 env "$@" python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/$n.log 2>&1; }
b base BEV_WARP_DIRECT=0 || exit $?
b direct BEV_WARP_DIRECT=1 || exit $?
b direct_occ4 BEV_WARP_DIRECT=1 BEV_WARP_OCC=4 || exit $?
b direct_p24 BEV_WARP_DIRECT=1 BEV_WARP_OCC=4 BEV_WARP_POOL_KB=24 || exit $?
b k5_base BEV_WARP_DIRECT=0 && true
timeout -k 10 120 env BEV_WARP_DIRECT=0 python bench.py --warp-only --views 16 --img 2160 3840 --steps 30 --warmup 3 --cpu-iters 0 > $O/k5_base.log 2>&1 || exit $?
timeout -k 10 120 env BEV_WARP_DIRECT=1 python bench.py --warp-only --views 16 --img 2160 3840 --steps 30 --warmup 3 --cpu-iters 0 > $O/k5_direct.log 2>&1 || exit $?
exit 0
