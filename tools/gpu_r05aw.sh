# Round 5 final-tree check: every GPU test, the smoke, the default bench line and the AMP training line.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
bash tools/gpu_r05_tests.sh $1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/train_step_bench.py --steps 12 --bevnet --amp > $O/train_amp.log 2>&1 || exit $?
exit 0
