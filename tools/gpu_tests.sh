#!/bin/bash
# One gpurun call: selected GPU tests (files / -k), then smoke().
#   gpurun --timeout 900 -- bash tools/gpu_tests.sh <tag> "<pytest args>"
TAG=${1:-r03}; ARGS=${2:-tests -m gpu}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 780 python -u -m pytest $ARGS -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] exit $rc"; grep -E "FAILED|Error|passed|failed" $OUT/pytest_gpu.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "[smoke] exit $rc"; tail -3 $OUT/smoke.log; exit $rc
