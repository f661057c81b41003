#!/bin/bash
# fused head-loss kernels: current build vs abold/ (the previous build), alternating processes
#   gpurun --timeout 600 -- 'bash tools/gpu_r05m.sh'
O=gpurun_out
R=$PWD
for i in 1 2; do
  DCLIP_LIB=$R/abold/libdclip.so DCLIP_TORCH_LIB=$R/abold/libdclip_torch.so timeout -k 10 120 python -u tools/headloss_probe.py 50 > $O/r05m_headloss_old_$i.log 2>&1 || exit $?
  timeout -k 10 120 python -u tools/headloss_probe.py 50 > $O/r05m_headloss_new_$i.log 2>&1 || exit $?
done
