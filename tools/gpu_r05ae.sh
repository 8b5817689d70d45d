# Round 5 pass ae: the head operand's dgrad computed for the BEV-feature channels alone -- AMP tests, the AMP step
# (x2) and its profile.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 500 --timeout-method thread tests/test_train_amp_gpu.py tests/test_head_gpu.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_amp_$r.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
exit 0
