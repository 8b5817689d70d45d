# Round GPU pass: GPU tests, the default bench line, and a rocprofv3 kernel-trace summary of the same command.
# usage (on the box): bash tools/gpu_round.sh <tag> [pytest -k expr]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-run}
K=${2:-}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1 || exit $?
exit 0
