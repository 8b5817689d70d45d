# Round 5 pass k: the v2 fused warp with all-views-at-once staging + the chunk-major output: warp / C-ABI /
# multi-GPU tests, A/B timings, and SQ counters of the old and new builds.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_warp_gpu.py tests/test_capi.py tests/test_dist_gpu.py > $O/warp_tests.log 2>&1 && timeout -k 10 120 python -u tools/warp_box_stats.py > $O/box_stats.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/warp_tests.log; [ $rc -ne 0 ] && exit $rc
ROUNDS=6 timeout -k 10 300 python -u tools/warp_ablate.py 0 cur sa 0nosa 0sad0 > $O/ab.txt 2>&1 || exit $?
VARIANTS="0 sa" bash tools/gpu_r05j.sh $1 || exit $?
exit 0
