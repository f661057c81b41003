set -o pipefail
cd /root/repo
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "work_conserving" > $O/pytest_gemm.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gemm.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_gemm_sched.py --rounds 7 > $O/ab_gemm_sched.log 2>&1; echo "ab rc=$?"
cat $O/ab_gemm_sched.log
