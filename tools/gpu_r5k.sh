# round 5 full run: GPU suite, grad-parity tables (-s), smoke, default bench, kernel stats
#   gpurun -- 'TAG=r5k bash tools/gpu_r5k.sh'
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5k}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest -s -q --timeout 300 --timeout-method thread tests/test_gpu_grad_parity.py > $O/grad_parity_tables.log 2>&1; echo "grad tables rc=$?"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
tail -1 $O/smoke.log
timeout -k 10 700 python -u bench.py > $O/bench.log 2> $O/bench.err || exit 4
cut -c1-300 $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 7 --warmup 3 --no-extras --no-fp16 --no-mode-r --cpu-baseline off --no-op-timing > $O/prof.log 2>&1 || exit 5
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/bench_kernel_stats.csv
t=$(find $O/prof -name "*kernel_trace.csv" | head -1); python tools/prof_summary.py $t --skip-marker attn_fwd3 --skip 36 --steps 7 --out $O/bench_steady_state.txt > /dev/null
rm -rf $O/prof
du -sh $O
