#!/bin/bash
# round 3: PMC of the dK/dV passes 5 vs 6 (same process), then the drop-in neck / heads tests + smoke
export TAG=r03c
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
P=1
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $R/$OUT/p$P -o run --output-format csv -- python3 $R/tools/ab_attn_opt.py 8 0 6 --rounds 1 > $R/$OUT/p$P.log 2>&1 || { echo "pmc pass $P failed"; tail -5 $R/$OUT/p$P.log; exit 1; }
  P=$((P+1))
done
cd $R
python tools/pmc_table.py $OUT/p1 $OUT/p2 > $OUT/pmc_table.txt 2>&1; grep -A18 "dkdv" $OUT/pmc_table.txt
bash tools/gpu_tests.sh $TAG "tests/test_gpu_dropin_heads.py tests/test_gpu_torch_ops.py tests/test_gpu_parity.py"
