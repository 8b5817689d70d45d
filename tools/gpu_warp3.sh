# Fused-warp pass: LDS atomic micro, every warp GPU test, warp-only bench of the default (v3) and v2 kernels, the
# full bench line, kernel traces of the full bench (default and one stream group), and the AMP BEVNet training step
# (timing + kernel trace).
# usage (on the box): [TESTS='tests/a.py tests/b.py'] bash tools/gpu_warp3.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
# (LDS atomic micro: profiles/r04c_lds_atomic_micro.txt)
timeout -k 10 1100 python -u -m pytest ${TESTS:-tests/test_warp_gpu.py} -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/warp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/warp_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/warp_bwd_micro.py > $O/bwd_micro.txt 2>&1 || exit $?
for k in rows dma; do
  timeout -k 10 300 python -u bench.py --warp-only --steps 30 --warmup 5 --cpu-iters 0 --warp-kernel $k > $O/warp_only_$k.log 2>&1 || exit $?
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-iters 0 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sg1 -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-iters 0 --stream-groups 1 > $O/prof_sg1.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/train_step_bench.py --bevnet --amp --steps 5 > $O/train_amp.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_train -o run -- python3 tools/train_step_bench.py --bevnet --amp --steps 2 --warmup 2 > $O/prof_train.log 2>&1 || exit $?
exit 0
