#!/bin/bash
# PMC passes over the final attention kernels (B=8, N=8193, H=12, bf16): MFMA busy, VALU/TRANS/LDS
# per MFMA, HBM bytes
OUT=gpurun_out/r04q; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/pmc_attn.sh $OUT/pmc || exit $?
python tools/pmc_table.py $(ls -d $OUT/pmc/p*/) > $OUT/table.txt 2>&1 || { tail -5 $OUT/table.txt; exit 1; }
rm -rf $OUT/pmc/p*/ 2>/dev/null
grep -A17 "fwd2_kernel\|dq2_kernel\|dkdv5_kernel" $OUT/table.txt | head -80
