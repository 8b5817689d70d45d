# Round 5 pass u: the ResNet stem on the split arithmetic (k_stem_x6) -- its accuracy test and the encoder parity
# tests, then the bench line with the split stem (default) and the exact-f32 stem (--stem-f32), alternating, and a
# kernel-trace summary of the default bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_conv_x6_gpu.py tests/test_backbone_gpu.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --cpu-iters 0 > $O/bench_x6stem_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --cpu-iters 0 --stem-f32 > $O/bench_f32stem_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/with_lib.py tools/_ab/libbev_presplit0.so bench.py --steps 30 --warmup 5 --cpu-iters 0 > $O/bench_presplit0_$r.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_train.py tests/test_train_amp_gpu.py > $O/tests_train.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests_train.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_amp.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
exit 0
