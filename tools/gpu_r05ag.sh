# Round 5 pass ag = ae + af: the head operand's dgrad for the BEV-feature channels alone (AMP / head tests, the AMP
# step x2 and its profile), then the HBM traffic of the default bench after the stem + max-pool fusion (the two PMC
# passes, reduced afterwards by tools/pmc_traffic.py).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 500 --timeout-method thread tests/test_head_operand_gpu.py tests/test_train_amp_gpu.py tests/test_head_gpu.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_amp_$r.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-iters 0 > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-iters 0 > $O/write.log 2>&1 || exit $?
exit 0
