# A/B of conv tile / staging variants over all ResNet-50 layers (tools/conv_micro.py).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
timeout -k 10 300 python3 tools/conv_micro.py --iters 10 --tiles 0 1 2 3 4 > gpurun_out/ab/xt.log 2>&1 || exit $?
