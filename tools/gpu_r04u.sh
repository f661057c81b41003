#!/bin/bash
# fast fp32 -> 16-bit weight transpose: kernel tests, timing, then a bench line
OUT=gpurun_out/r04u; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "transpose" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -u tools/transpose_probe.py > $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
cat $OUT/probe.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '"metric"' $OUT/bench.log | cut -c1-200
