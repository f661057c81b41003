#!/bin/bash
# One gpurun call: the GPU test suite (optionally a -k selection), then (if it passed) the bench.
#   gpurun --timeout 1200 -- bash tools/gpu_suite.sh <tag> [pytest -k expr] [bench args...]
TAG=${1:-r02}; K=${2:-}
shift 2 2>/dev/null
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 720 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] exit $rc"; grep -E "FAILED|Error|passed|failed" $OUT/pytest_gpu.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 3 "$@" > $OUT/bench.log 2>&1
rc=$?; echo "[bench] exit $rc"; tail -c 2500 $OUT/bench.log; exit $rc
