set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/phases; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 -k "units or full_size or fused" > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for w in 2 1; do
  BEV_WARP_WOCC=$w BEV_WARP_DEBUG=64 timeout -k 10 120 python tools/warp_phases.py > $O/ph_w$w.log 2>&1 || exit $?
  BEV_WARP_WOCC=$w BEV_WARP_DEBUG=78 timeout -k 10 120 python tools/warp_phases.py > $O/ph_w${w}_skel.log 2>&1 || exit $?
  BEV_WARP_WOCC=$w timeout -k 10 120 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/bench_w$w.log 2>&1 || exit $?
done
for d in 2 4 8; do
  BEV_WARP_DEBUG=$d timeout -k 10 120 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/bench_dbg$d.log 2>&1 || exit $?
done
exit 0
