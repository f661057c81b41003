#!/bin/bash
# Round-2 profile set in one gpurun call:
#   1. rocprofv3 kernel-trace stats of the bench step (mode F, bf16, B = 8)
#   2. FETCH_SIZE / WRITE_SIZE passes (separate runs) over the attention probe -> HBM traffic of
#      the backward's kernels
#   3. the NT / TN token GEMMs against torch.mm (hipBLASLt)
#   gpurun --timeout 900 -- bash tools/gpu_prof_r02.sh <tag>
TAG=${1:-r02prof}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/bench_trace.log 2>&1 || exit $?
f=$(find $OUT/trace -name "run_kernel_stats.csv" | head -1); cp $f $OUT/bench_kernel_stats.csv
cut -c1-150 $OUT/bench_kernel_stats.csv | head -25
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/f1 -o run --output-format csv -- python tools/attn_probe.py 2 > $OUT/f1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/f2 -o run --output-format csv -- python tools/attn_probe.py 2 > $OUT/f2.log 2>&1 || exit $?
D=$(find $OUT/f1 $OUT/f2 -name run_counter_collection.csv -exec dirname {} \;)
for k in attn_bwd_dq2_kernel attn_bwd_dkdv5_kernel attn_bwd_row0 attn_fwd2_kernel; do
  python tools/pmc_traffic.py $D --kernel $k --algorithmic 1 > $OUT/traffic_$k.txt 2>&1
  echo "== $k"; cat $OUT/traffic_$k.txt
done
timeout -k 10 240 python tools/gemm_vs_blas.py 5 > $OUT/gemm_vs_blas.log 2>&1 || exit $?
cat $OUT/gemm_vs_blas.log
