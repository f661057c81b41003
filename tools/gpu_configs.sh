#!/bin/bash
# BASELINE configs [3] / [4], inference lines and the dK/dV variant A/B on one box:
#   gpurun --timeout 1500 -- 'TAG=r03f bash tools/gpu_configs.sh'
OUT=gpurun_out/${TAG:-cfg}; mkdir -p $OUT
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 420 python bench.py --no-mode-r --no-fp16 --cpu-baseline off "$@" > $OUT/$name.log 2>&1 || exit $?; echo "== $name"; grep "^{" $OUT/$name.log | cut -c1-300; }
timeout -k 10 120 tools/mfma_clock 20000 > $OUT/mfma_clock.log 2>&1 || exit $?; cat $OUT/mfma_clock.log
run headline_dkdv5 --steps 10 --warmup 3
DCLIP_OPTIONS=8=6 run headline_dkdv6 --steps 10 --warmup 3
run vitl14_dkdv5 --arch vitl14 --steps 3 --warmup 2
DCLIP_OPTIONS=8=6 run vitl14_dkdv6 --arch vitl14 --steps 3 --warmup 2
run fp8_train --attn-fp8 --steps 5 --warmup 2
run infer_bf16 --infer --steps 10 --warmup 3
run infer_fp8 --infer --attn-fp8 --steps 10 --warmup 3
