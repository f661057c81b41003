# persistent GEMM K-loop with fragment reads one group ahead (DCLIP_OPT_GEMM_KLOOP 1): per-GEMM and step A/B
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 200 python3 tools/ab_gemm_tail.py 7 17 0,1 > $O/ab_gemm_kloop.log 2>&1 || exit 5
grep -v amdgpu.ids $O/ab_gemm_kloop.log
timeout -k 10 600 python3 tools/ab_flag.py opt:17 0 1 --rounds 4 --steps 10 > $O/ab_step_kloop.log 2>&1 || exit 6
tail -3 $O/ab_step_kloop.log
