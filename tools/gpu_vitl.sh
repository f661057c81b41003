#!/bin/bash
# One gpurun call: the ViT-L/14 + patchify GPU tests, then a ViT-L/14 bench line.
#   gpurun --timeout 900 -- bash tools/gpu_vitl.sh <tag>
TAG=${1:-vitl}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "vitl14 or im2col" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] exit $rc"; grep -E "PASSED|FAILED|Error|passed|failed" $OUT/pytest_gpu.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --arch vitl14 --steps ${STEPS:-4} --warmup 2 --no-mode-r --cpu-baseline off \
  > $OUT/bench.log 2>&1
rc=$?; echo "[bench] exit $rc"; tail -c 2500 $OUT/bench.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$VITB" ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-mode-r --cpu-baseline off > $OUT/bench_vitb.log 2>&1
  rc=$?; echo "[bench vitb] exit $rc"; tail -c 600 $OUT/bench_vitb.log
fi
exit $rc
