# Backbone tests (incl. dual conv) + conv micro (fused tails) + warp PMC passes + HBM bytes for both rooflines.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider > $O/warp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/warp_tests.log; [ $rc -ne 0 ] && exit $rc
BEV_WARP_POOL_KB=8 timeout -k 10 600 python -m pytest tests/test_warp_gpu.py -q -x -p no:cacheprovider -k "full_size or fused" > $O/warp_tests_pool8.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/warp_tests_pool8.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/bench_v2.log 2>&1 || exit $?
BEV_WARP_V1=1 timeout -k 10 300 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/bench_v1.log 2>&1 || exit $?
BEV_WARP_OCC=2 timeout -k 10 300 python bench.py --warp-only --steps 50 --warmup 5 --cpu-iters 0 > $O/bench_v2_occ2.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/conv_micro.py l1.0.ds l1.0.c3 l1.0.tail l2.0.ds l2.1.c3 l2.0.tail --iters 10 > $O/micro.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d $O/w$i -o run -- python3 $R/bench.py --warp-only --steps 3 --warmup 1 --cpu-iters 0 > $O/w$i.log 2>&1 || exit $?
done
for pmc in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d $O/b$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-iters 0 > $O/b$i.log 2>&1 || exit $?
done
exit 0
