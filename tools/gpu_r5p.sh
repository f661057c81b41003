# streaming-store rule (DCLIP_OPT_GEMM_EPI 0) vs none (3) vs all (2): per-GEMM and step A/B, plus GEMM tests
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5p}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > $O/pytest_gemm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gemm.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 tools/ab_gemm_tail.py 7 10 0,3,2 > $O/ab_gemm_epi.log 2>&1 || exit 5
grep -v amdgpu.ids $O/ab_gemm_epi.log
timeout -k 10 700 python3 tools/ab_flag.py opt:10 0 3 --rounds 5 --steps 10 > $O/ab_step_epi.log 2>&1 || exit 6
tail -3 $O/ab_step_epi.log
timeout -k 10 500 python3 tools/ab_flag.py opt:10 0 3 --rounds 3 --steps 10 --fp16 > $O/ab_step_epi_fp16.log 2>&1 || exit 7
tail -3 $O/ab_step_epi_fp16.log
