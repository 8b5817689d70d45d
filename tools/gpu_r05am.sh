# Round 5 pass am: BatchNorm streaming passes with batched row loads (BN_U rows in flight, compile-time activation):
# the BN / training tests, then the AMP step alternating with the previous bev_bn.hip (tools/_ab/libbev_bnold.so),
# then the kernel statistics of the new step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q -p no:cacheprovider --timeout 500 --timeout-method thread -m gpu tests/test_train.py tests/test_train_amp_gpu.py tests/test_effnet.py tests/test_bevnet_gpu.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 8 --bevnet --amp > $O/train_new_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/with_lib.py tools/_ab/libbev_bnold.so tools/train_step_bench.py --steps 8 --bevnet --amp > $O/train_old_$r.log 2>&1 || exit $?
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof_old -o run -- python3 tools/with_lib.py tools/_ab/libbev_bnold.so tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof_old.log 2>&1 || exit $?
exit 0
