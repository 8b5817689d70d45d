# Round 5 pass al: the target construction joins the loss graph (host targets): tests, the AMP step alternating
# default / --no-loss-graph / the round's previous behaviour, then the ordered kernel trace of one default step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 500 --timeout-method thread -m gpu tests/test_targets.py tests/test_bevnet_gpu.py tests/test_train_amp_gpu.py tests/test_train.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 8 --bevnet --amp > $O/train_new_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 8 --bevnet --amp --no-loss-graph > $O/train_nograph_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 8 --bevnet --amp --no-loss-graph --eager-decode --device-targets > $O/train_old_$r.log 2>&1 || exit $?
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/ttrace -o run -- python3 tools/train_step_bench.py --steps 1 --warmup 1 --bevnet --amp > $O/ttrace.log 2>&1 || exit $?
exit 0
