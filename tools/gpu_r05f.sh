# Round 5 pass f: the fused warp's skeleton (ablation variants 31 / 30 / 14 and the full kernel): wave cycles,
# waits and instruction mix per wave, one rocprofv3 --pmc pass per variant.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
P="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for b in ${VARIANTS:-31 30 14 0}; do
  ROUNDS=2 timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/v$b -o run -- python3 tools/warp_ablate.py $b > $O/v$b.log 2>&1 || exit $?
done
exit 0
