set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ph2; mkdir -p $O
for o in 4 2; do
  BEV_WARP_OCC=$o BEV_WARP_DEBUG=64 timeout -k 10 120 python tools/warp_phases_v2.py > $O/occ$o.log 2>&1 || exit $?
  BEV_WARP_OCC=$o BEV_WARP_DEBUG=79 timeout -k 10 120 python tools/warp_phases_v2.py > $O/occ${o}_skel.log 2>&1 || exit $?
done
exit 0
