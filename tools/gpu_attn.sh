#!/bin/bash
# One gpurun call: attention kernel tests (optional -k filter), then the option A/B timing.
#   gpurun -- bash tools/gpu_attn.sh <tag> "<pytest -k expr>" "8=0" "8=1" ...
TAG=${1:-attn}; K=${2:-attention}
shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
rc=$?; echo "[pytest] exit $rc"; tail -5 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_opt_ab.py "$@" > $OUT/ab.log 2>&1
rc=$?; echo "[ab] exit $rc"; cat $OUT/ab.log; exit $rc
