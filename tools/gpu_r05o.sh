#!/bin/bash
# eager weight-copy refresh: its tests, then the step A/B (on / off) in one process
#   gpurun --timeout 900 -- 'bash tools/gpu_r05o.sh'
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "weight_refresh or conv3x3_weight or upsample" -q --timeout 120 --timeout-method thread > $O/r05o_pytest.log 2>&1 || { tail -30 $O/r05o_pytest.log; exit 1; }
tail -1 $O/r05o_pytest.log
timeout -k 10 400 python -u tools/ab_flag.py ops.EAGER_WEIGHT_REFRESH True False --rounds 3 --steps 10 > $O/r05o_ab_refresh.log 2>&1 || exit $?
tail -2 $O/r05o_ab_refresh.log
