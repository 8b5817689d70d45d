# Round 5 pass c: VALU / LDS counters of each fused-warp ablation variant (tools/warp_ablate.sh builds), one
# rocprofv3 --pmc pass per variant and counter group, so each part's share of the VALU cycles can be read off.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
P="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for b in ${VARIANTS:-0 1 2 4 8 16 24}; do
  ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/v$b -o run -- python3 tools/warp_ablate.py $b > $O/v$b.log 2>&1 || exit $?
done
exit 0
