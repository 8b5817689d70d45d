set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/k5; mkdir -p $O
timeout -k 10 300 python bench.py --warp-only --views 16 --img 2160 3840 --steps 30 --warmup 3 --cpu-iters 0 > $O/warp_k5.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --warp-only --channels 128 --steps 30 --warmup 3 --cpu-iters 0 > $O/warp_c128.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --views 16 --img 2160 3840 --steps 3 --warmup 1 --cpu-iters 0 > $O/full_k5.log 2>&1 || exit $?
exit 0
