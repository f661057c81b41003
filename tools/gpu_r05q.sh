#!/bin/bash
# kernel traces of 5 bf16 and 5 fp16 steps: where the fp16 step's extra time goes (GPU idle gaps
# vs kernel time)
#   gpurun --timeout 900 -- 'bash tools/gpu_r05q.sh'
O=$PWD/gpurun_out/r05q; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
for m in bf16 fp16; do
  F=""; [ $m = fp16 ] && F="--fp16"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$m -o run -- python3 $R/tools/step_runner.py $F --warmup 3 --steps 5 > $O/$m.log 2>&1) || exit $?
  f=$(find $O/$m -name "*kernel_trace.csv" | head -1)
  python3 tools/gap_summary.py $f --skip 36 --steps 5 > $O/gaps_$m.txt || exit $?
  python3 tools/prof_summary.py $f --skip-marker attn_fwd2 --skip 36 --steps 5 --out $O/kernels_$m.txt > /dev/null || exit $?
  head -30 $O/gaps_$m.txt
done
