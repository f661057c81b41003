# K-loop read-ahead rule (DCLIP_OPT_GEMM_KLOOP 0) vs none (2): per-GEMM and step A/B (bf16, fp16)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 300 python3 tools/ab_gemm_tail.py 7 17 0,2 > $O/ab_gemm_kloop.log 2>&1 || exit 5
grep -v amdgpu.ids $O/ab_gemm_kloop.log | tail -12
timeout -k 10 600 python3 tools/ab_flag.py opt:17 0 2 --rounds 4 --steps 10 > $O/ab_step_kloop.log 2>&1 || exit 6
tail -2 $O/ab_step_kloop.log
timeout -k 10 500 python3 tools/ab_flag.py opt:17 0 2 --rounds 3 --steps 10 --fp16 > $O/ab_step_kloop_fp16.log 2>&1 || exit 7
tail -2 $O/ab_step_kloop_fp16.log
