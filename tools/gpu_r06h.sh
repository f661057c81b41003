#!/bin/bash
# packed fp32 softmax arithmetic (v_pk_mul_f32 / v_pk_add_f32) in the attention passes: one-process
# A/B against the previous build (abx/libdclip_base.so), bf16 and fp16
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 240 python -u tools/ab_attn.py -r 9 $R/abx/libdclip_base.so $R/abx/libdclip_pk.so > gpurun_out/r06h_ab_pk_bf16.log 2>&1 &&
timeout -k 10 240 python -u tools/ab_attn.py -r 9 --fp16 $R/abx/libdclip_base.so $R/abx/libdclip_pk.so > gpurun_out/r06h_ab_pk_fp16.log 2>&1
