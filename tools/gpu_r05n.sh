# Round 5 pass n: taps-ahead A/B (K2), then the full pass (tests, smoke, bench, profiles, K5 / K4 lines, training).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
ROUNDS=5 timeout -k 10 300 python -u tools/warp_ablate.py 0 ta0 ta1 ta6 > $O/ab_taps.txt 2>&1 || exit $?
TRAIN=1 bash tools/gpu_r05_full.sh $1
