# fp16 16-bit LN-backward inputs (ABI 6): LN / fp16 / grad-parity tests, the default bench, then the GEMM-vs-hipBLASLt trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5m}; mkdir -p $O
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm" > $O/pytest_ln.log 2>&1
rc=$?; echo "pytest ln rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_ln.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_native_abi.py tests/test_gpu_fp16.py \
  tests/test_gpu_grad_parity.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 700 python -u bench.py > $O/bench.log 2> $O/bench.err || exit 4
cut -c1-400 $O/bench.log
python3 -c "
import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1])
print('bf16', d['value'], d['ms_per_step'], 'fp16', d.get('fp16',{}).get('value'), 'ratio', d.get('fp16',{}).get('value',0)/d['value'])"
timeout -k 10 200 python3 tools/gemm_vs_blas.py 5 > $O/gemm_vs_blas.log 2>&1 || exit 5
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/gemm_vs_blas.py 2 > $O/traced.log 2>&1 || exit 6
f=$(find $O/p -name "*kernel_stats.csv" | head -1)
cp $f $O/gemm_kernel_stats.csv; rm -rf $O/p
