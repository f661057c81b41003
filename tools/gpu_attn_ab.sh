#!/bin/bash
OUT=gpurun_out/r01d; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -k "attention" --timeout 120 --timeout-method thread > $OUT/pytest_attn.log 2>&1; rc=$?
echo "[pytest] $rc"; tail -4 $OUT/pytest_attn.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/attn_fwd_ab.py 7 > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
