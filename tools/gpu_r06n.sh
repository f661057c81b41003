#!/bin/bash
# HBM traffic of the LayerNorm backward forms in the bf16 train step (FETCH_SIZE / WRITE_SIZE in
# separate rocprofv3 --pmc passes over tools/step_runner.py, 1 warm-up + 1 step)
OUT=gpurun_out/r06n_pmc_ln
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv \
  -- python tools/step_runner.py --warmup 1 --steps 1 > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv \
  -- python tools/step_runner.py --warmup 1 --steps 1 > $OUT/write.log 2>&1 || exit $?
for p in fetch write; do f=$(find $OUT/$p -name run_counter_collection.csv | head -1); cp "$f" $OUT/$p/; done
# ln_1 with the read-out add (906 MB algorithmic), ln_2 with a bf16 dy and the lp copy (805 MB)
python tools/pmc_traffic.py $OUT/fetch $OUT/write --kernel "3, false, true>" --algorithmic 906e6 --out $OUT/traffic_ln_bwd_add.json > /dev/null || exit $?
python tools/pmc_traffic.py $OUT/fetch $OUT/write --kernel "ln_bwd_fast<bool _Accum, 3, false, false>" --algorithmic 805e6 --out $OUT/traffic_ln_bwd_lp.json > /dev/null || exit $?
echo "[pmc ln traffic] done"; cat $OUT/traffic_*.json
