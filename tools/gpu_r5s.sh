# element-wise census of the bench step (which copies / adds, on which stream)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-extras --no-fp16 --no-mode-r --cpu-baseline off --no-op-timing > $O/prof.log 2>&1 || exit 5
t=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/copy_census.py $t 7 > $O/census.txt; cat $O/census.txt
head -1 $t > $O/trace_head.csv
rm -rf $O/prof
