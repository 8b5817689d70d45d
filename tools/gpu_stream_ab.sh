# A/B of the ResNet stream-group split: bench.py per (groups, offset), one line each.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_backbone_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k stream_groups > $O/t.log 2>&1 || exit 1
for go in "1 0" "2 0" "2 1" "2 2" "2 3" "3 0" "3 1" "3 3"; do
  set -- $go
  timeout -k 10 200 python -u bench.py --cpu-iters 0 --steps 40 --stream-groups $1 --stream-offset $2 > $O/b_$1_$2.log 2>&1 || exit 1
  echo "$1 $2 $(tail -1 $O/b_$1_$2.log)" >> $O/ab.txt
done
exit 0
