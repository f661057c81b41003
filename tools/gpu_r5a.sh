set -o pipefail
cd /root/repo
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_grad_parity.py tests/test_gpu_fp16.py tests/test_gpu_torch_ops.py > gpurun_out/r5a_pytest.log 2>&1
rc=$?
echo "rc1=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm or readout or ln_ or LayerNorm" > gpurun_out/r5a_pytest_ln.log 2>&1
echo "rc2=$?"
