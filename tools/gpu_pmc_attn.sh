#!/bin/bash
# PMC passes over the attention probe (default kernels) + table:  gpurun -- bash tools/gpu_pmc_attn.sh <tag>
OUT=gpurun_out/${1:-pmc}; mkdir -p $OUT
bash tools/pmc_attn.sh $OUT/pmc_attn; rc=$?
python tools/pmc_table.py $(ls -d $OUT/pmc_attn/p*/) > $OUT/pmc_attn/table.txt 2>&1; cat $OUT/pmc_attn/table.txt | grep -A25 "^attn_fwd2"
exit $rc
