#!/bin/bash
# MFMA-shape clock diagnostic: real kernels vs the 16x16x32-substituted diag build, alternately
OUT=gpurun_out/r04b; mkdir -p $OUT
export TMPDIR=/tmp
L=denseclip_vit_multimodal_amd
for i in 1 2 3; do
  timeout -k 10 120 python tools/mfma_shape_diag.py $L/libdclip.so 20 >> $OUT/diag.log 2>&1 || { tail $OUT/diag.log; exit 1; }
  timeout -k 10 120 python tools/mfma_shape_diag.py $L/libdclip_diag.so 20 >> $OUT/diag.log 2>&1 || { tail $OUT/diag.log; exit 1; }
done
grep -v amdgpu.ids $OUT/diag.log
