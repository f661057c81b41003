#!/bin/bash
# re-measure the kept kernel-variant options on the current tree (one process per sweep)
O=gpurun_out
timeout -k 10 200 python -u tools/ab_attn_opt.py 8 0 5 --rounds 7 > $O/r05y_ab_bwd_block.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ab_attn_opt.py 5 0 128 --rounds 7 > $O/r05y_ab_dkdv_qs.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ab_attn_opt.py 1 0 4 --rounds 7 > $O/r05y_ab_dq_waves.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ab_attn_opt.py 0 0 4 --rounds 7 --fwd > $O/r05y_ab_fwd_waves.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_gemm_opt.py 0 7 9 5 > $O/r05y_ab_gemm_tile.log 2>&1 || exit $?
grep -h "med\|total\|ms" $O/r05y_ab_*.log | grep -v "equal" | head -60
