set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/tbox; mkdir -p $O
BEV_WARP_TBOX=1 timeout -k 10 600 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 -k "fused" > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
b() { n=$1; shift; timeout -k 10 120 env "$@" python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/$n.log 2>&1; }
b base BEV_WARP_OCC=4 || exit $?
b tbox BEV_WARP_OCC=4 BEV_WARP_TBOX=1 || exit $?
b base2 BEV_WARP_OCC=2 || exit $?
b tbox2 BEV_WARP_OCC=2 BEV_WARP_TBOX=1 || exit $?
b tbox_dbg15 BEV_WARP_TBOX=1 BEV_WARP_DEBUG=15 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 bench.py --warp-only --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
exit 0
