set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/xcd; mkdir -p $O
BEV_CONV_XCD=1 timeout -k 10 600 python -u -m pytest tests/test_backbone_gpu.py -x -q -p no:cacheprovider --timeout 300 > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
BEV_CONV_XCD=0 timeout -k 10 600 python3 tools/conv_micro.py --iters 10 > $O/micro0.log 2>&1 || exit $?
BEV_CONV_XCD=1 timeout -k 10 600 python3 tools/conv_micro.py --iters 10 > $O/micro1.log 2>&1 || exit $?
BEV_CONV_XCD=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-iters 0 > $O/bench0.log 2>&1 || exit $?
BEV_CONV_XCD=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-iters 0 > $O/bench1.log 2>&1 || exit $?
exit 0
