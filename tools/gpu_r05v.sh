#!/bin/bash
# 64-row dQ pass: parity against the default, then the in-process A/B of the backward
#   gpurun --timeout 900 -- 'bash tools/gpu_r05v.sh'
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "dq_rows64 or dkdv6_matches or bwd_full_length" -q --timeout 200 --timeout-method thread > $O/r05v_pytest.log 2>&1 || { tail -30 $O/r05v_pytest.log; exit 1; }
tail -1 $O/r05v_pytest.log
timeout -k 10 300 python -u tools/ab_attn_opt.py 14 0 64 --rounds 7 > $O/r05v_ab_dq_rows.log 2>&1 || exit $?
tail -4 $O/r05v_ab_dq_rows.log
