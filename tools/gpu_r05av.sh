# Round 5 pass av: AMP step, native focal loss vs --torch-focal, three alternating rounds of 12 steps.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 12 --bevnet --amp > $O/train_new_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 12 --bevnet --amp --torch-focal > $O/train_old_$r.log 2>&1 || exit $?
done
exit 0
