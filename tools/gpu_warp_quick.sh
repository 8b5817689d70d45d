# First contact with a new warp kernel: small fixtures only, short limits.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "test_fused_nhwc_kernels and (w3_v3 or w7_tiny or w2_b2)" > $O/quick.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/quick.log; exit $rc
