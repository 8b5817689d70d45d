# Config lines other than the default bench: EfficientNet-B3 (configs[3]) and the camera-shard K5 path (configs[4])
# at world 1, each its own bench.py JSON line.
# usage (on the box): bash tools/gpu_lines.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u bench.py --backbone efficientnet_b3 --steps 20 --warmup 5 --cpu-iters 0 > $O/effb3.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --camera-shard --steps 10 --warmup 3 --cpu-iters 0 > $O/cam.log 2>&1 || exit $?
exit 0
