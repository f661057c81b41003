#!/bin/bash
# row-mean / score-map rewrite: kernel + model parity tests, then a profiled bench
OUT=gpurun_out/r04f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "score or row_mean or context or vitb16" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 2 > $OUT/bench_trace.log 2>&1 || exit $?
f=$(find $OUT/trace -name "run_kernel_stats.csv" | head -1); cp $f $OUT/kstats.csv
grep -E "score_map|row_mean" $OUT/kstats.csv | cut -d, -f1-4
grep '"metric"' $OUT/bench_trace.log | cut -c1-150
