#!/bin/bash
# BASELINE configs [3] / [4] and inference lines on one box:
#   gpurun --timeout 1100 -- bash tools/gpu_configs.sh <tag>
TAG=${1:-r02cfg}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 420 python bench.py --no-mode-r --cpu-baseline off "$@" > $OUT/$name.log 2>&1 || exit $?; echo "== $name"; grep "^{" $OUT/$name.log | cut -c1-330; }
run fp8_train --attn-fp8 --steps 5 --warmup 2
run vitl14_train --arch vitl14 --steps 3 --warmup 2
run infer_bf16 --infer --steps 10 --warmup 3
run infer_fp8 --infer --attn-fp8 --steps 10 --warmup 3
