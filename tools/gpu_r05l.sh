#!/bin/bash
# round-4 probes: fused head-loss tests + old/new timing, host-sync probe, dq2 priority A/B,
# text-path precision probe
#   gpurun --timeout 900 -- 'bash tools/gpu_r05l.sh'
O=gpurun_out
R=$PWD
timeout -k 10 60 ./abold/dq_atomic_probe > $O/r05l_dq_atomic_probe.log 2>&1 || exit $?
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k "upsample" -q --timeout 120 --timeout-method thread > $O/r05l_pytest_headloss.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/headloss_probe.py 20 > $O/r05l_headloss_new.log 2>&1 || exit $?
DCLIP_LIB=$R/abold/libdclip.so DCLIP_TORCH_LIB=$R/abold/libdclip_torch.so timeout -k 10 120 python -u tools/headloss_probe.py 20 > $O/r05l_headloss_old.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/sync_probe.py > $O/r05l_sync_probe.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ab_attn.py -r 7 $R/denseclip_vit_multimodal_amd/libdclip.so $R/abold/libdclip_prio.so > $O/r05l_ab_dq2_prio.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/text_probe.py 3 10 > $O/r05l_text_probe.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ab_wgrad_opt.py 0 2 3 4 > $O/r05l_ab_wgrad_opt.log 2>&1 || exit $?
