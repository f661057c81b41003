#!/bin/bash
# epilogue constants prefetched at tile start: GEMM parity tests + timing (bias epilogue) vs hipBLASLt
OUT=gpurun_out/r04e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm and (6 or 7 or 8 or 9)" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python tools/gemm_vs_blas.py 5 > $OUT/blas6.log 2>&1 || { tail $OUT/blas6.log; exit 1; }
grep -v amdgpu $OUT/blas6.log
