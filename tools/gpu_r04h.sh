#!/bin/bash
# forward reference update tied into negm's registers: attention tests, then A/B timing vs the previous build
OUT=gpurun_out/r04h; mkdir -p $OUT
export TMPDIR=/tmp
L=denseclip_vit_multimodal_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "attn_bwd or attention_bwd or bwd" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2 3; do
  timeout -k 10 120 python tools/mfma_shape_diag.py $L/libdclip_base.so 20 >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  timeout -k 10 120 python tools/mfma_shape_diag.py $L/libdclip.so 20 >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
done
grep -v amdgpu $OUT/ab.log
