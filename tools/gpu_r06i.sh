#!/bin/bash
# attn_fwd3 row sums from the packed 16-bit P (v_dot2): one-process A/B against the previous build,
# bf16 and fp16, then the attention tests on the new build
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 240 python -u tools/ab_attn.py -r 9 $R/abx/libdclip_base.so $R/abx/libdclip_dot2.so > gpurun_out/r06i_ab_dot2_bf16.log 2>&1 &&
timeout -k 10 240 python -u tools/ab_attn.py -r 9 --fp16 $R/abx/libdclip_base.so $R/abx/libdclip_dot2.so > gpurun_out/r06i_ab_dot2_fp16.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "attention or attn" > gpurun_out/r06i_pytest_attn.log 2>&1
