set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/train; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_effnet.py -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; exit $rc
