# Round 5 pass z2: the training tests with the mask-bytes recorders, the AMP step with and without mask bytes, then the
# fused warp's channel split (WARP_CK=32: two workgroups per tile, 3 / 4 / 5 per CU) A/B against the product build and
# the split variant's warp parity tests.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread tests/test_train.py tests/test_train_amp_gpu.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_mask_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp --no-mask-bytes > $O/train_nomask_$r.log 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/warp_prod_$r.log 2>&1 || exit $?
  for v in ck32o3 ck32o4 ck32o5; do
    timeout -k 10 200 python -u tools/with_lib.py tools/_ab/libbev_$v.so bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/warp_${v}_$r.log 2>&1 || exit $?
  done
done
timeout -k 10 600 python -u tools/with_lib.py tools/_ab/libbev_ck32o4.so tools/run_pytest.py tests/test_warp_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/warp_tests_ck32o4.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/warp_tests_ck32o4.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
exit 0
