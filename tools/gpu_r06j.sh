#!/bin/bash
# bf16 LayerNorm-backward inputs from the dX GEMMs (ops.LN_DY_LP): train-step A/B in one process,
# then the whole GPU suite with the flag on (the default)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_flag.py ops.LN_DY_LP True False --rounds 4 --steps 8 > gpurun_out/r06j_ab_ln_dy_lp.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06j_pytest_gpu.log 2>&1
