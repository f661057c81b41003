# new M-tail kernel: tail tests + LN tests, A/B timing, rocprof of the A/B (tail kernel durations)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5n}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "tail or gemm" > $O/pytest_gemm.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gemm.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 tools/ab_gemm_tail.py 7 > $O/ab_gemm_tail.log 2>&1 || exit 5
cat $O/ab_gemm_tail.log | grep -v amdgpu.ids
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/ab_gemm_tail.py 2 > $O/traced.log 2>&1 || exit 6
f=$(find $O/p -name "*kernel_stats.csv" | head -1)
cp $f $O/ab_kernel_stats.csv; rm -rf $O/p
grep -i tail $O/ab_kernel_stats.csv | cut -d, -f1-4 | cut -c1-200
