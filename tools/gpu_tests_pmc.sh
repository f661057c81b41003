#!/bin/bash
# One gpurun call: the GPU test suite, then the attention PMC passes (HBM traffic for the
# bench's roofline object).   gpurun --timeout 900 -- bash tools/gpu_tests_pmc.sh <tag>
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] exit $rc" | tee -a $OUT/steps.log; tail -3 $OUT/pytest_gpu.log
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit $rc; fi
bash tools/pmc_attn.sh $OUT/pmc_attn; rc=$?; echo "[pmc] exit $rc" | tee -a $OUT/steps.log
python tools/pmc_table.py $OUT/pmc_attn/p* > $OUT/pmc_attn/table.txt 2>&1; cat $OUT/pmc_attn/table.txt
exit $rc
