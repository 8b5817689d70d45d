# Round 5 pass az: the native gaussian radius joining the native losses: tests, then the AMP step
# alternating with --torch-loss (three rounds of 12 steps).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 500 --timeout-method thread -m gpu tests/test_targets.py tests/test_capi.py tests/test_bevnet_gpu.py tests/test_train_amp_gpu.py tests/test_train.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 12 --bevnet --amp > $O/train_new_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 12 --bevnet --amp --torch-loss > $O/train_old_$r.log 2>&1 || exit $?
done
exit 0
