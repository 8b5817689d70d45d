# Round 5 pass aa: the stem with the max-pool fused into its epilogue -- its bit-identity tests, the split-conv and
# backbone / BEVNet parity tests through the eval chain, then the bench with and without it (alternating) + profile.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "stem_pool" tests/test_conv_x6_gpu.py > $O/tests_stem_pool.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests_stem_pool.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_conv_x6_gpu.py tests/test_backbone_gpu.py tests/test_bevnet_gpu.py tests/test_train.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --cpu-iters 0 > $O/bench_pool_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --cpu-iters 0 --no-stem-pool > $O/bench_nopool_$r.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-iters 0 --stream-groups 1 > $O/prof.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_amp.log 2>&1 || exit $?
exit 0
