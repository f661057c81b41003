# round 5: full GPU suite, smoke, default bench, kernel stats, a DDP (world size 1) kernel trace reduced
# on the box (raw traces deleted: gpurun_out must stay under 64 MiB), the GEMM tile-walk A/B
#   gpurun -- 'TAG=r5d bash tools/gpu_r5c.sh'
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${TAG:-r5c}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
tail -1 $O/smoke.log
timeout -k 10 300 python -u tools/ab_gemm_sched.py --rounds 5 > $O/ab_gemm_sched.log 2>&1 || exit 7
tail -8 $O/ab_gemm_sched.log
timeout -k 10 700 python -u bench.py > $O/bench.log 2> $O/bench.err || exit 4
cut -c1-300 $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 7 --warmup 3 --no-extras --no-fp16 --no-mode-r --cpu-baseline off --no-op-timing > $O/prof.log 2>&1 || exit 5
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/bench_kernel_stats.csv
t=$(find $O/prof -name "*kernel_trace.csv" | head -1); python tools/prof_summary.py $t --skip-marker attn_fwd --skip 36 --steps 7 --out $O/bench_steady_state.txt > /dev/null
rm -rf $O/prof
MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ddp -o run -- python3 bench.py --ddp --steps 3 --warmup 2 --no-extras --no-fp16 --no-mode-r --cpu-baseline off --no-op-timing > $O/prof_ddp.log 2>&1 || exit 6
t=$(find $O/prof_ddp -name "*kernel_trace.csv" | head -1); python tools/ddp_trace.py $t --out $O/ddp_trace.txt | tail -5
f=$(find $O/prof_ddp -name "*kernel_stats.csv" | head -1); cp $f $O/ddp_kernel_stats.csv
rm -rf $O/prof_ddp
du -sh $O
