# Round-5 end-of-round pass, part 2: the default bench line and its rocprofv3 kernel-trace summary, the camera-shard
# (K5) and EfficientNet-B3 (K4) lines, and the AMP training line (K3) with its profile.
# usage (on the box): bash tools/gpu_r05_lines.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --camera-shard --steps 10 --warmup 2 --cpu-iters 0 > $O/cam.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --backbone efficientnet_b3 --steps 20 --warmup 3 --cpu-iters 0 > $O/effb3.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_amp.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
exit 0
