#!/bin/bash
# GEMM epilogue order A/B: pre-session gemm.hip / HEAD (column pairs outer) / rows outer, real epilogues
OUT=gpurun_out/r04l; mkdir -p $OUT
export TMPDIR=/tmp
L=denseclip_vit_multimodal_amd
for r in 1 2; do
for v in pre head new; do
  cp $L/libdclip_$v.so $L/libdclip.so
  echo "== $v" >> $OUT/epi.log
  timeout -k 10 200 python tools/gemm_epi_bench.py 3 >> $OUT/epi.log 2>&1 || { tail $OUT/epi.log; exit 1; }
done
done
cp $L/libdclip_new.so $L/libdclip.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -v amdgpu $OUT/epi.log
