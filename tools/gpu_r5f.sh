# round 5: kernel stats of the default step, the DDP (world size 1) bucket placement, and the
# inference step with bf16 vs fp8 attention (raw traces reduced on the box and deleted)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5f}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 7 --warmup 3 --no-extras --no-fp16 --no-mode-r --cpu-baseline off --no-op-timing > $O/prof.log 2>&1 || exit 5
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/bench_kernel_stats.csv
t=$(find $O/prof -name "*kernel_trace.csv" | head -1); python tools/prof_summary.py $t --skip-marker attn_fwd --skip 36 --steps 7 --out $O/bench_steady_state.txt > /dev/null
rm -rf $O/prof
MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ddp -o run -- python3 bench.py --ddp --steps 3 --warmup 2 --no-extras --no-fp16 --no-mode-r --cpu-baseline off --no-op-timing > $O/prof_ddp.log 2>&1 || exit 6
t=$(find $O/prof_ddp -name "*kernel_trace.csv" | head -1); python tools/ddp_trace.py $t --out $O/ddp_trace.txt | tail -4
f=$(find $O/prof_ddp -name "*kernel_stats.csv" | head -1); cp $f $O/ddp_kernel_stats.csv
rm -rf $O/prof_ddp
for m in bf16 fp8; do
  extra=""; [ $m = fp8 ] && extra="--attn-fp8"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_inf_$m -o run -- python3 bench.py --infer $extra --steps 10 --warmup 3 --no-extras --cpu-baseline off --no-op-timing > $O/prof_inf_$m.log 2>&1 || exit 7
  t=$(find $O/prof_inf_$m -name "*kernel_trace.csv" | head -1); python tools/prof_summary.py $t --skip-marker im2col --skip 3 --steps 10 --out $O/infer_${m}_steady_state.txt > /dev/null
  rm -rf $O/prof_inf_$m
  grep '"metric"' $O/prof_inf_$m.log | cut -c1-200
done
du -sh $O
