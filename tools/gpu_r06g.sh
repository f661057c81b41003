#!/bin/bash
# conv weight-gradient 128 x 256 tile: parity tests, then the train step A/B (default vs wide tile)
# under a kernel trace so both kernels' averages come from one process
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "conv3x3_wgrad" > gpurun_out/r06g_pytest.log 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r06g_prof -o run -- \
  python3 tools/ab_flag.py opt:16 0 256 --rounds 3 --steps 8 > gpurun_out/r06g_ab.log 2>&1
