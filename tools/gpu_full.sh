#!/bin/bash
# the whole GPU suite, smoke(), the default bench line, and a rocprofv3 kernel-stats run of the bench step
#   TAG=r03d gpurun --timeout 1200 -- bash tools/gpu_full.sh
OUT=gpurun_out/${TAG:-r03d}; mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '"metric"' $OUT/bench.log | cut -c1-400
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --steps 5 --warmup 2 --no-mode-r --no-fp16 --cpu-baseline off > $R/$OUT/prof.log 2>&1 || { tail -20 $R/$OUT/prof.log; exit 1; }
cd $R; f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 $f | head -25
