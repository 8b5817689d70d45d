# Round 5 pass g: the v2 fused warp with scalar row LDS-DMA staging and the fp32 mean: warp GPU tests (bit-exact vs
# the oracle), then A/B timings of the variants (old kernel "0", new "n0", 8 x 32 tiles, 4 workgroups per CU).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_warp_gpu.py tests/test_capi.py tests/test_dist_gpu.py > $O/warp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/warp_tests.log; [ $rc -ne 0 ] && exit $rc
ROUNDS=5 timeout -k 10 300 python -u tools/warp_ablate.py 0 n0 n0t8 n0o4 n0t8o4 n0d0 n0m0 > $O/ab.txt 2>&1 || exit $?
exit 0
