# Round-5 warp evidence: SQ / LDS counters of the fused warp inside the bench pipeline (7 cams, 1080p, batch 2)
# and on the camera-shard line (16 cams, 4K), each PMC group in a run of its own, the HBM traffic of the
# camera-shard launch (FETCH_SIZE / WRITE_SIZE passes), kernel traces of both, and the default bench line.
# usage (on the box): bash tools/gpu_r05_warp_pmc.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --cpu-iters 0 > $O/bench.log 2>&1 || exit $?
for mode in pipe cam; do
  X="--steps 6 --warmup 2 --cpu-iters 0"; [ $mode = cam ] && X="--camera-shard --steps 4 --warmup 1 --cpu-iters 0"
  timeout -s KILL 170 rocprofv3 --pmc $P1 --output-format csv -d $O/${mode}_p1 -o run -- python3 bench.py $X > $O/${mode}_p1.log 2>&1 || exit $?
  timeout -s KILL 170 rocprofv3 --pmc $P2 --output-format csv -d $O/${mode}_p2 -o run -- python3 bench.py $X > $O/${mode}_p2.log 2>&1 || exit $?
  timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${mode}_kt -o run -- python3 bench.py $X > $O/${mode}_kt.log 2>&1 || exit $?
done
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cam_fetch -o run -- python3 bench.py --camera-shard --steps 3 --warmup 1 --cpu-iters 0 > $O/cam_fetch.log 2>&1 || exit $?
timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cam_write -o run -- python3 bench.py --camera-shard --steps 3 --warmup 1 --cpu-iters 0 > $O/cam_write.log 2>&1 || exit $?
exit 0
