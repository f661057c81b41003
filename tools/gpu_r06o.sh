#!/bin/bash
# fp16 read-out gradient fold (dclip_layernorm_bwd_scaled_add): the fp16 suite + the fold tests, then
# the fp16 train-step A/B in one process
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "test_gpu_fp16 or layernorm_bwd_add or readout_grad_fold or add_readout" > gpurun_out/r06o_pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_flag.py ops.FOLD_READOUT_GRAD True False --rounds 4 --steps 8 --fp16 > gpurun_out/r06o_ab_fold_fp16.log 2>&1
