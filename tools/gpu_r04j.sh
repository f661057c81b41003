#!/bin/bash
# fp16 dS pre-scale folded into the register fragments: fp16 / attention tests, A/B timing + bitwise fingerprint
OUT=gpurun_out/r04j; mkdir -p $OUT
export TMPDIR=/tmp
L=denseclip_vit_multimodal_amd
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp16.py -k "attn or fp16" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  for dt in 1 2; do
    timeout -k 10 120 python tools/mfma_shape_diag.py $L/libdclip_base.so 15 $dt >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
    timeout -k 10 120 python tools/mfma_shape_diag.py $L/libdclip.so 15 $dt >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  done
done
grep -v amdgpu $OUT/ab.log
