# persistent GEMM epilogue with streaming stores (DCLIP_OPT_GEMM_EPI 2): per-GEMM A/B, then the step A/B
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5o}; mkdir -p $O
timeout -k 10 200 python3 tools/ab_gemm_tail.py 7 10 0,2 > $O/ab_gemm_epi.log 2>&1 || exit 5
grep -v amdgpu.ids $O/ab_gemm_epi.log
timeout -k 10 500 python3 tools/ab_flag.py opt:10 0 2 --rounds 3 --steps 10 > $O/ab_step_epi.log 2>&1 || exit 6
tail -6 $O/ab_step_epi.log
