#!/bin/bash
# persistent GEMM variants (DCLIP_OPT_GEMM_TILE 6..9): parity tests, then timing vs hipBLASLt
OUT=gpurun_out/r04c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm and (6 or 7 or 8 or 9)" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for t in 6 7 8 9; do
  DCLIP_OPTIONS=3=$t timeout -k 10 200 python tools/gemm_vs_blas.py 5 > $OUT/blas$t.log 2>&1 || { tail $OUT/blas$t.log; exit 1; }
  echo "--- tile $t"; grep "NT" $OUT/blas$t.log
done
