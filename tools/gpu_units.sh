# Fused warp variants: parity (all fixtures, forced pools), timing per variant, ablations.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/units; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 -k "units or full_size or fused" > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
b() { timeout -k 10 120 env "$@" python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0; }
b BEV_WARP_WOCC=2 > $O/w2.log 2>&1 || exit $?
b BEV_WARP_WOCC=3 > $O/w3.log 2>&1 || exit $?
b BEV_WARP_WOCC=4 > $O/w4.log 2>&1 || exit $?
for d in 2 4 8 14; do b BEV_WARP_WOCC=2 BEV_WARP_DEBUG=$d > $O/w2_dbg$d.log 2>&1 || exit $?; done
exit 0
