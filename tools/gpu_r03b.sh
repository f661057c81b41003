#!/bin/bash
# round 3, first GPU call: the dK/dV variant 6 (test + A/B + trace), then the drop-in neck / heads tests + smoke
export TAG=r03b
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "dkdv6" -x -v --timeout 120 --timeout-method thread > $OUT/pytest_dkdv6.log 2>&1
rc=$?; echo "[dkdv6 tests] exit $rc"; grep -E "PASS|FAIL|Error|passed|failed" $OUT/pytest_dkdv6.log | tail -20; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_dkdv6.sh || exit $?
bash tools/gpu_tests.sh $TAG "tests/test_gpu_dropin_heads.py tests/test_gpu_torch_ops.py tests/test_gpu_parity.py"
