#!/bin/bash
# Kernel-trace stats + two PMC passes over tools/attn_probe.py for the given bwd-block variants.
#   gpurun -- bash tools/gpu_prof_attn.sh <tag> 0,1,2
TAG=${1:-prof}; V=${2:-0}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python tools/attn_probe.py 3 $V > $OUT/trace.log 2>&1 || exit $?
f=$(find $OUT/trace -name "run_kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
cut -c1-160 $OUT/kernel_stats.csv | head -14
P=1
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$P -o run --output-format csv -- python tools/attn_probe.py 2 $V > $OUT/p$P.log 2>&1 || exit $?
  P=$((P+1))
done
python tools/pmc_table.py $OUT/p1 $OUT/p2 > $OUT/table.txt 2>&1
grep -A17 "dkdv\|dq2" $OUT/table.txt
