#!/bin/bash
# One gpurun call: the headline bench (mode F + R + CPU baseline), the inference benches
# (bf16 and fp8 attention, BASELINE configs[4]), the ViT-L/14 train step (configs[3]) and rocprofv3 kernel stats of the headline
# and of the fp8 inference.  Stops at the first step that does not exit cleanly.
#   gpurun --timeout 1200 -- bash tools/gpu_configs.sh <tag>
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# step <name> <log> <command...>: runs the command with its output in <log>, stops on failure
step() { local name=$1 log=$2; shift 2; "$@" > "$log" 2>&1; local rc=$?; echo "[$name] exit $rc" | tee -a $OUT/steps.log; [ $rc -eq 0 ] || exit $rc; }
step bench $OUT/bench.log timeout -k 10 420 python bench.py --steps 10 --warmup 3
tail -1 $OUT/bench.log
step infer $OUT/bench_infer.log timeout -k 10 300 python bench.py --infer --steps 10 --warmup 3
tail -1 $OUT/bench_infer.log
step infer_fp8 $OUT/bench_infer_fp8.log timeout -k 10 300 python bench.py --attn-fp8 --steps 10 --warmup 3
tail -1 $OUT/bench_infer_fp8.log
step vitl14 $OUT/bench_vitl14.log timeout -k 10 400 python bench.py --arch vitl14 --steps 4 --warmup 2 --no-mode-r --cpu-baseline off
tail -1 $OUT/bench_vitl14.log
step prof $OUT/bench_prof.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python bench.py --steps 3 --warmup 2 --no-mode-r --cpu-baseline off
step prof_fp8 $OUT/bench_prof_fp8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run --output-format csv -- \
  python bench.py --attn-fp8 --steps 3 --warmup 2
