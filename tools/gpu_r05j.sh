# Round 5 pass j: SQ counters of fused-warp builds (per-variant rocprofv3 --pmc passes: instruction mix, then
# VALU / LDS busy), tools/warp_ablate.py launches.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for b in ${VARIANTS:-0 cur 128}; do
  ROUNDS=2 timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/p1/v$b -o run -- python3 tools/warp_ablate.py $b > $O/p1_v$b.log 2>&1 || exit $?
  ROUNDS=2 timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $O/p2/v$b -o run -- python3 tools/warp_ablate.py $b > $O/p2_v$b.log 2>&1 || exit $?
done
exit 0
