#!/bin/bash
# PMC passes over a GEMM driver:  bash tools/pmc_gemm.sh out_dir
#   PROBE: the python arguments (default: the weight-gradient A/B, asm K-loop 0 vs builtin 5)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_gemm}
mkdir -p $OUT
PROBE=${PROBE:-tools/ab_wgrad_opt.py 0 5}
run() { timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/p$PASS -o run --output-format csv -- python3 $PROBE > $OUT/p$PASS.log 2>&1; PASS=$((PASS+1)); }
PASS=1
run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM
run FETCH_SIZE
run TCC_HIT_sum TCC_MISS_sum
