# fp16 vs bf16 train-step kernel traces: per-kernel totals and GPU idle gaps (reduced on the box)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5j; mkdir -p $O
for m in bf16 fp16; do
  extra=""; [ $m = fp16 ] && extra="--fp16"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_$m -o run -- python3 tools/step_runner.py $extra --warmup 3 --steps 5 > $O/$m.log 2>&1 || exit 3
  t=$(find $O/p_$m -name "*kernel_trace.csv" | head -1)
  python tools/prof_summary.py $t --skip-marker attn_fwd3 --skip 36 --steps 5 --out $O/${m}_steady_state.txt > /dev/null
  (cd tools && python gap_summary.py ../$t --marker attn_fwd3 --skip 36 --steps 5 --top 20) > $O/${m}_gaps.txt 2>&1
  rm -rf $O/p_$m
  head -3 $O/${m}_steady_state.txt; head -4 $O/${m}_gaps.txt
done
