#!/bin/bash
# attention forward kernel variants: per-launch A/B (bf16, f16), then the train step A/B
O=gpurun_out
timeout -k 10 200 python -u tools/ab_attn_opt.py 6 0 3 --rounds 11 --fwd > $O/r05w_ab_fwd_bf16.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ab_attn_opt.py 6 0 3 --rounds 11 --fwd --dt f16 > $O/r05w_ab_fwd_f16.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_flag.py opt:6 0 3 --rounds 3 --steps 10 > $O/r05w_ab_fwd_step.log 2>&1 || exit $?
grep -h "med\|median" $O/r05w_ab_fwd_bf16.log $O/r05w_ab_fwd_f16.log $O/r05w_ab_fwd_step.log
