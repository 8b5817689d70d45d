# Round 5 pass l: VALU issue-rate microbenchmark; fused-warp A/B on the bench geometry (K2) and the camera-shard
# geometry (K5: 16 cams 4K, SUM) -- default build, stage-all off, 2 workgroups per CU with larger LDS pools.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
timeout -k 10 60 ./tools/valu_rate_micro > $O/valu_rate.txt 2>&1 || exit $?
ROUNDS=5 timeout -k 10 300 python -u tools/warp_ablate.py 0 cur t_sa t_nosa t_o2 > $O/ab_k2.txt 2>&1 || exit $?
GEOM=k5 ROUNDS=4 timeout -k 10 300 python -u tools/warp_ablate.py 0 t_sa t_nosa t_o2b_p72 > $O/ab_k5.txt 2>&1 || exit $?
exit 0
