# Round 5 pass ar: (1) the graphed-loss check (tools/loss_graph_check.py, 3 seeds); (2) the fused warp's channels-last
# output after the store fix (no spills): warp / C-ABI tests, smoke, bench alternating with --warp-nchw.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
for s in 0 1 2; do
  timeout -k 10 200 python -u tools/loss_graph_check.py $s > $O/loss_check_$s.log 2>&1 || exit $?
done
bash tools/gpu_r05ap.sh $1
