#!/bin/bash
# kernel stats of BASELINE config [3] (ViT-L/14 train step, ragged CLS-split attention) and the fp8 inference line
OUT=gpurun_out/r04s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --arch vitl14 --no-mode-r --cpu-baseline off --steps 3 --warmup 1 > $OUT/vitl14_trace.log 2>&1 || exit 1
f=$(find $OUT/trace -name "run_kernel_stats.csv" | head -1); cp $f $OUT/vitl14_kstats.csv; rm -rf $OUT/trace
head -8 $OUT/vitl14_kstats.csv | cut -d, -f1-4 | cut -c1-160
timeout -k 10 300 python bench.py --infer --attn-fp8 --no-mode-r --cpu-baseline off --steps 10 --warmup 3 > $OUT/infer_fp8.log 2>&1 || exit 1
grep "^{" $OUT/infer_fp8.log | cut -c1-200
