#!/bin/bash
# PMC passes over the attention backward A/B (tools/ab_attn_bwd1.py, one process, arms $ARMS), one
# rocprofv3 run per counter group:  gpurun -- 'TAG=r6o ARMS=0,10 bash tools/pmc_bwd1.sh'
#   -> python tools/pmc_table.py gpurun_out/$TAG/p*
set -e
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc_bwd1}
mkdir -p $OUT
cd /tmp
run() { timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/p$PASS -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ab_attn_bwd1.py --rounds 1 --reps 2 --arms ${ARMS:-0,10} > $OUT/p$PASS.log 2>&1; echo "[pass $PASS] ok"; PASS=$((PASS+1)); }
PASS=1
run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32
run FETCH_SIZE
run WRITE_SIZE
cd $GRAFT_REPO_ROOT && python3 tools/pmc_table.py $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 > $OUT/pmc_table.txt && grep -A17 "attn_bwd" $OUT/pmc_table.txt | head -120
