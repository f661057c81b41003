#!/bin/bash
# One gpurun call: GPU test suite, then (if it passed) a short bench.
#   gpurun --timeout 900 -- bash tools/gpu_tests_bench.sh <tag> [pytest -k expr]
TAG=${1:-r01}; K=${2:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] exit $rc"; grep -E "FAILED|Error|passed|failed" $OUT/pytest_gpu.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python bench.py --steps ${STEPS:-5} --warmup 2 --no-mode-r --cpu-baseline off > $OUT/bench.log 2>&1
rc=$?; echo "[bench] exit $rc"; tail -c 1500 $OUT/bench.log; exit $rc
