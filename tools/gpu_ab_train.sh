# Parity tests, then the fp16 conv micro and the AMP training step, product library vs variant builds
# (tools/build_variant.sh), alternating, then the product's training profile.
#   bash tools/gpu_ab_train.sh <tag> <variant>[,<variant>...] "<pytest files>"
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
VS=$(echo $2 | tr ',' ' ')
if [ -n "${3:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread $3 > $O/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 200 python -u tools/conv_h16_micro.py --wgrad > $O/micro_prod.log 2>&1 || exit $?
for v in $VS; do
  timeout -k 10 200 python -u tools/with_lib.py tools/_ab/libbev_$v.so tools/conv_h16_micro.py --wgrad > $O/micro_$v.log 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_prod_$r.log 2>&1 || exit $?
  for v in $VS; do
    timeout -k 10 300 python -u tools/with_lib.py tools/_ab/libbev_$v.so tools/train_step_bench.py --steps 5 --bevnet --amp > $O/train_${v}_$r.log 2>&1 || exit $?
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1 || exit $?
exit 0
