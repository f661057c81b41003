# CLS row pass beside the forward's main pass (DCLIP_OPT_ATTN_ROW0 0 vs 1): tests, step A/B (ABBA), inference A/B, rocprof overlap
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5z; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "row0_beside or attention or attn" tests/test_gpu_torch_ops.py tests/test_gpu_parity.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 tools/ab_flag.py opt:18 0 1 --rounds 4 --steps 10 > $O/ab_step_row0.log 2>&1 || exit 6
tail -2 $O/ab_step_row0.log
