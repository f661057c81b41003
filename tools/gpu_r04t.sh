#!/bin/bash
# PMC passes over the token GEMMs at the bench shape (tools/gemm_probe.py), final binaries:
# the weight-gradient (TN) kernel's wait / LDS / MFMA split for the next-round GEMM lever
OUT=gpurun_out/r04t; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/pmc_gemm.sh $OUT/pmc || exit $?
python tools/pmc_table.py $(ls -d $OUT/pmc/p*/) > $OUT/table.txt 2>&1 || { tail -5 $OUT/table.txt; exit 1; }
rm -rf $OUT/pmc/p*/ 2>/dev/null
grep -A20 "gemm_tn_big" $OUT/table.txt | head -60
