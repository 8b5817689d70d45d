# Warp A/B: parity of the fused warp tests, then warp-only timings per variant (env pairs in $@ style list below).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/wab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
b() { n=$1; shift; timeout -k 10 120 env "$@" python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/$n.log 2>&1; }
b occ4 BEV_WARP_OCC=4 || exit $?
b occ2 BEV_WARP_OCC=2 || exit $?
b occ2_p96 BEV_WARP_OCC=2 BEV_WARP_POOL_KB=96 || exit $?
b occ2_p64 BEV_WARP_OCC=2 BEV_WARP_POOL_KB=64 || exit $?
for d in 1 2 8 15; do b occ2_dbg$d BEV_WARP_OCC=2 BEV_WARP_DEBUG=$d || exit $?; done
exit 0
