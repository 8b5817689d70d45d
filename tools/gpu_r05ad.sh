# Round 5 pass ad: training tests (max-pool argmax forms), the AMP step with / without the forward argmax bytes
# (alternating), then the end-of-round lines (tools/gpu_r05_lines.sh) on the same box.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_train.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_arg_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp --no-pool-arg > $O/train_noarg_$r.log 2>&1 || exit $?
done
bash tools/gpu_r05_lines.sh $1
