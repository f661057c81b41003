#!/bin/bash
# final tree: full GPU suite, smoke(), headline bench + rocprof kernel stats, fp16 / ViT-L / fp8 / inference lines
OUT=gpurun_out/r04o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
run() { name=$1; t=$2; shift 2; timeout -k 10 $t python bench.py "$@" > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }; echo "== $name"; grep "^{" $OUT/$name.log | cut -c1-200; }
run bench 420 --steps 10 --warmup 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-mode-r --cpu-baseline off > $OUT/bench_trace.log 2>&1 || exit 1
f=$(find $OUT/trace -name "run_kernel_stats.csv" | head -1); cp $f $OUT/kstats.csv; rm -rf $OUT/trace
run bench_fp16 300 --dtype fp16 --no-mode-r --cpu-baseline off --steps 10 --warmup 3
run vitl14_train 420 --arch vitl14 --no-mode-r --cpu-baseline off --steps 3 --warmup 2
run fp8_train 300 --attn-fp8 --no-mode-r --cpu-baseline off --steps 5 --warmup 2
run infer_bf16 300 --infer --no-mode-r --cpu-baseline off --steps 10 --warmup 3
