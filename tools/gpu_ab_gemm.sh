#!/bin/bash
# A/B of dclip_gemm tile variants in one process: gpurun -- bash tools/gpu_ab_gemm.sh <tag> <tiles...>
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python tools/gemm_variants.py 7 "$@" > $OUT/gemm_variants.log 2>&1; rc=$?
cat $OUT/gemm_variants.log; exit $rc
