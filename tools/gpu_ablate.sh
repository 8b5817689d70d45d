# Backbone parity (stem kernel), warp ablation timings, full bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/abl; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_backbone_gpu.py -q -x -p no:cacheprovider > $O/bb_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/bb_tests.log; [ $rc -ne 0 ] && exit $rc
BEV_WARP_WIDE=1 timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider -k "full_size or fused" > $O/warp_wide_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/warp_wide_tests.log; [ $rc -ne 0 ] && exit $rc
BEV_WARP_WIDE=1 timeout -k 10 300 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/warp_wide.log 2>&1 || exit $?
for d in 0 1 2 4 8 6 14 15; do
  BEV_WARP_DEBUG=$d timeout -k 10 300 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/warp_dbg$d.log 2>&1 || exit $?
done
timeout -k 10 600 python bench.py --cpu-iters 0 > $O/bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
exit 0
