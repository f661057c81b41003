#!/bin/bash
# session measurements: headline bench (bf16, mode R, CPU baseline), fp16 line, rocprof kernel stats,
# BASELINE configs [3] / [4] and inference lines
OUT=gpurun_out/r04k; mkdir -p $OUT
export TMPDIR=/tmp
run() { name=$1; t=$2; shift 2; timeout -k 10 $t python bench.py "$@" > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }; echo "== $name"; grep "^{" $OUT/$name.log | cut -c1-260; }
run bench 420 --steps 10 --warmup 3
run bench_fp16 300 --dtype fp16 --no-mode-r --cpu-baseline off --steps 10 --warmup 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-mode-r --cpu-baseline off > $OUT/bench_trace.log 2>&1 || exit 1
f=$(find $OUT/trace -name "run_kernel_stats.csv" | head -1); cp $f $OUT/kstats.csv; rm -rf $OUT/trace
run fp8_train 300 --attn-fp8 --no-mode-r --cpu-baseline off --steps 5 --warmup 2
run vitl14_train 420 --arch vitl14 --no-mode-r --cpu-baseline off --steps 3 --warmup 2
run infer_bf16 300 --infer --no-mode-r --cpu-baseline off --steps 10 --warmup 3
run infer_fp8 300 --infer --attn-fp8 --no-mode-r --cpu-baseline off --steps 10 --warmup 3
