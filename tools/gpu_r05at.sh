# Round 5 final pass: every GPU test and the smoke, then the end-of-round lines (bench + kernel trace, K5,
# EfficientNet-B3, AMP training step + kernel trace).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/gpu_r05_tests.sh $1 || exit $?
bash tools/gpu_r05_lines.sh $1
