# Round 5 pass ao: the store-pattern microbenchmark with the channels-last (NHWC) output patterns, then the
# end-of-round lines of this tree (bench + kernel trace, K5, EfficientNet-B3, AMP training step + kernel trace).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 120 ./tools/store_pattern_micro > $O/store_micro.txt 2>&1 || exit $?
bash tools/gpu_r05_lines.sh $1
