#!/bin/bash
# deferred dQ MFMAs: parity, then the in-process A/B of the backward (bf16, f16)
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "dq_variants" -q --timeout 200 --timeout-method thread > $O/r05z_pytest.log 2>&1 || { tail -30 $O/r05z_pytest.log; exit 1; }
tail -1 $O/r05z_pytest.log
timeout -k 10 200 python -u tools/ab_attn_opt.py 15 0 1 --rounds 11 > $O/r05z_ab_defer_bf16.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ab_attn_opt.py 15 0 1 --rounds 11 --dt f16 > $O/r05z_ab_defer_f16.log 2>&1 || exit $?
grep -h "med\|equal" $O/r05z_ab_defer_*.log
