# Round 5 pass p: whole-line staging loads in k_conv_h16b (H16B_LINES) and the 16-B head operand kernels --
# parity tests, the AMP training step A/B against the H16B_LINES=0 variant, and the training profile.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread tests/test_head_operand_gpu.py "tests/test_warp_gpu.py::test_fused_max_backward_vs_torch_autograd" tests/test_conv_h16_gpu.py tests/test_train_amp_gpu.py tests/test_train.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/conv_h16_micro.py --wgrad > $O/micro_lines1.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/with_lib.py tools/_ab/libbev_lines0.so tools/conv_h16_micro.py --wgrad > $O/micro_lines0.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_lines1_$r.log 2>&1 || exit $?
  timeout -k 10 300 python -u tools/with_lib.py tools/_ab/libbev_lines0.so tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_lines0_$r.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
exit 0
