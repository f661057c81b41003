OUT=gpurun_out/r03d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "weight_grad or gemm_tn" tests/test_gpu_fp16.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 2 > $OUT/bench_trace.log 2>&1 || exit $?
f=$(find $OUT/trace -name "run_kernel_stats.csv" | head -1); cp $f $OUT/kstats.csv
grep -E "gemm_tn|colsum" $OUT/kstats.csv | cut -c1-200
tail -1 $OUT/bench_trace.log | cut -c1-300
