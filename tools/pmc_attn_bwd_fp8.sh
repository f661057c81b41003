#!/bin/bash
# PMC passes over tools/ab_attn_bwd_fp8.py (dkdv6 vs dkdv8 in one process; one rocprofv3 run per counter group)
#   bash tools/pmc_attn_bwd_fp8.sh [out_dir]  ->  python tools/pmc_table.py out_dir/p*
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_bwd_fp8}
mkdir -p $OUT
run() { timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/p$PASS -o run --output-format csv -- python tools/ab_attn_bwd_fp8.py --rounds 1 --reps 3 > $OUT/p$PASS.log 2>&1; PASS=$((PASS+1)); }
PASS=1
run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32
