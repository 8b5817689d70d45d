# Round 5 pass x: per-layer counters of the inference trunk (single stream group, so launches are attributable):
# MFMA busy / waits / VALU / LDS / L2 hit / HBM bytes per conv launch of one bench step -> tools/trunk_layer_table.py
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
X="--steps 2 --warmup 1 --cpu-iters 0 --stream-groups 1"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
P3="SQ_WAVES TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P4="SQ_WAVES WRITE_SIZE"
P5="SQ_WAVES FETCH_SIZE"
n=1
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $O/p$n -o run -- python3 bench.py $X > $O/p$n.log 2>&1 || exit $?
  n=$((n+1))
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py $X > $O/kt.log 2>&1 || exit $?
exit 0
