#!/bin/bash
# HBM traffic of the attention passes at the benchmark shape: FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 --pmc passes over tools/attn_probe.py (2 fwd + bwd reps), then per-kernel
# bytes per launch by tools/pmc_traffic.py.
#   bash tools/pmc_attn_traffic.sh [out_dir]
OUT=${1:-gpurun_out/pmc_attn_traffic}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv \
  -- python tools/attn_probe.py 2 > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv \
  -- python tools/attn_probe.py 2 > $OUT/write.log 2>&1 || exit $?
# rocprofv3 nests its csv one level down (<dir>/<host>/<pid>/run_*.csv): flatten for pmc_traffic.py
for p in fetch write; do f=$(find $OUT/$p -name run_counter_collection.csv | head -1); cp "$f" $OUT/$p/; done
for k in attn_bwd_dq2_kernel attn_bwd_dkdv6_kernel attn_bwd_row0 attn_fwd3_kernel attn_row0; do
  python tools/pmc_traffic.py $OUT/fetch $OUT/write --kernel $k --algorithmic 1 --out $OUT/traffic_$k.json > /dev/null || exit $?
done
echo "[pmc traffic] done"; grep -h '"hbm_bytes_per_launch"\|"kernel"' $OUT/traffic_*.json
