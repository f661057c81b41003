#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/r02i
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "score_map" > gpurun_out/r02i/pytest.log 2>&1
rc=$?; echo "[pytest] $rc"; tail -3 gpurun_out/r02i/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_prof_attn.sh r02i 1,3 > gpurun_out/r02i/prof.log 2>&1; rc=$?; echo "[prof] $rc"; exit $rc
