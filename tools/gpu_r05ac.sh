# Round 5 pass ac: the training max-pool with the forward's argmax bytes -- training tests, then the AMP step with
# and without it (--no-pool-arg), alternating, and its profile.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 600 --timeout-method thread tests/test_train.py tests/test_train_amp_gpu.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_arg_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp --no-pool-arg > $O/train_noarg_$r.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
exit 0
