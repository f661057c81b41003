#!/bin/bash
# PMC passes over tools/attn_probe.py (one rocprofv3 run per counter group).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_attn}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python tools/attn_probe.py 2 > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 -d $OUT/p2 -o run --output-format csv -- python tools/attn_probe.py 2 > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/p3 -o run --output-format csv -- python tools/attn_probe.py 2 > $OUT/p3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/p4 -o run --output-format csv -- python tools/attn_probe.py 2 > $OUT/p4.log 2>&1
ls -R $OUT | head -30
