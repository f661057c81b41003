#!/bin/bash
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "text or context or ddp" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '"metric"' $OUT/bench.log | cut -c1-220
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 2 > $OUT/bench_trace.log 2>&1 || exit $?
f=$(find $OUT/trace -name "run_kernel_stats.csv" | head -1); cp $f $OUT/kstats.csv
grep '"metric"' $OUT/bench_trace.log | cut -c1-220
