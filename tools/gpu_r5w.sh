# ABBA re-check of the streaming-store rule (opt 10: 0 vs 3) and the K-loop read-ahead rule (opt 17: 0 vs 2),
# per GEMM and per step, plus an A/A control of the step A/B
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 300 python3 tools/ab_gemm_tail.py 8 17 0,2 > $O/ab_gemm_kloop.log 2>&1 || exit 5
grep -v amdgpu.ids $O/ab_gemm_kloop.log | tail -12
timeout -k 10 300 python3 tools/ab_gemm_tail.py 8 10 0,3 > $O/ab_gemm_nts.log 2>&1 || exit 5
grep -v amdgpu.ids $O/ab_gemm_nts.log | tail -12
timeout -k 10 600 python3 tools/ab_flag.py opt:17 0 2 --rounds 4 --steps 10 > $O/ab_step_kloop.log 2>&1 || exit 6
tail -2 $O/ab_step_kloop.log
timeout -k 10 600 python3 tools/ab_flag.py opt:10 0 3 --rounds 4 --steps 10 > $O/ab_step_nts.log 2>&1 || exit 7
tail -2 $O/ab_step_nts.log
timeout -k 10 600 python3 tools/ab_flag.py opt:5 0 0 --rounds 4 --steps 10 > $O/ab_step_aa.log 2>&1 || exit 8
tail -4 $O/ab_step_aa.log
