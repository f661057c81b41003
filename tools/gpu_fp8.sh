#!/bin/bash
# One gpurun call: the fp8 attention tests, then inference bench lines (bf16 attention, fp8 attention)
#   gpurun --timeout 900 -- bash tools/gpu_fp8.sh <tag>
TAG=${1:-fp8}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -v -s --timeout 200 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] exit $rc"; grep -E "^E  .{0,200}|PASSED|FAILED|passed|failed" $OUT/pytest_gpu.log | cut -c1-250 | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --infer --steps 10 --warmup 3 > $OUT/bench_infer_bf16.log 2>&1
rc=$?; echo "[bench infer bf16] exit $rc"; tail -c 1500 $OUT/bench_infer_bf16.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --attn-fp8 --steps 10 --warmup 3 > $OUT/bench_infer_fp8.log 2>&1
rc=$?; echo "[bench infer fp8] exit $rc"; tail -c 1500 $OUT/bench_infer_fp8.log
exit $rc
