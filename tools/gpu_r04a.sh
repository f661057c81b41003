#!/bin/bash
# session baseline: bench + hipBLASLt kernel names/durations for the token GEMM shapes
OUT=gpurun_out/r04a; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '"metric"' $OUT/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/blas -o run --output-format csv -- python tools/gemm_vs_blas.py 3 > $OUT/blas.log 2>&1 || exit $?
f=$(find $OUT/blas -name "run_kernel_stats.csv" | head -1); cp $f $OUT/blas_kstats.csv
cat $OUT/blas.log | grep -v amdgpu.ids
