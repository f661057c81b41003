set -o pipefail
cd /root/repo
O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "captured or text" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|Error" $O/pytest.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --no-mode-r --no-fp16 --cpu-baseline off --no-op-timing > $O/bench.log 2> $O/bench.err; echo "bench rc=$?"
grep "\[bench" $O/bench.err
