# Round 5 pass o: BEVNet / training tests after the native head-operand assembly, then the training line + profile.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 1100 --timeout-method thread tests/test_bevnet_gpu.py tests/test_head_gpu.py tests/test_train_amp_gpu.py tests/test_train.py tests/test_data_wildtrack.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_amp.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
exit 0
