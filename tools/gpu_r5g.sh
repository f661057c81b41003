set -o pipefail
cd /root/repo
O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "captured" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|Error" $O/pytest.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --no-mode-r --no-fp16 --cpu-baseline off --no-op-timing > $O/bench.log 2> $O/bench.err; echo "bench rc=$?"
grep "\[bench" $O/bench.err
timeout -k 10 300 python -u tools/glue_probe.py fp16 > $O/glue_fp16.log 2>&1; echo "glue fp16 rc=$?"
timeout -k 10 300 python -u tools/glue_probe.py bf16 > $O/glue_bf16.log 2>&1; echo "glue bf16 rc=$?"
