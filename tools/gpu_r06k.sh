#!/bin/bash
# read-out gradient folded into the next block's ln_1 backward (ops.FOLD_READOUT_GRAD): parity tests,
# then the train-step A/B in one process
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "layernorm_bwd_add or readout_grad_fold or add_readout_cast" > gpurun_out/r06k_pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_flag.py ops.FOLD_READOUT_GRAD True False --rounds 4 --steps 8 > gpurun_out/r06k_ab_fold.log 2>&1
