#!/bin/bash
# CLS-split attention at ragged N (ViT-L/14's 10659): kernel tests (all attention), A/B timing at the headline shape
OUT=gpurun_out/r04n; mkdir -p $OUT
export TMPDIR=/tmp
L=denseclip_vit_multimodal_amd
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "attn or attention" > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 120 python tools/mfma_shape_diag.py $L/libdclip_base.so 15 >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  timeout -k 10 120 python tools/mfma_shape_diag.py $L/libdclip.so 15 >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
done
grep -v amdgpu $OUT/ab.log
timeout -k 10 420 python bench.py --arch vitl14 --no-mode-r --cpu-baseline off --steps 3 --warmup 2 > $OUT/vitl14.log 2>&1 || { tail -5 $OUT/vitl14.log; exit 1; }
grep "^{" $OUT/vitl14.log | cut -c1-200
