#!/bin/bash
# the whole GPU suite, smoke(), the default bench line, and a rocprofv3 kernel-stats run of the bench step
#   gpurun --timeout 1500 -- 'TAG=r03e bash tools/gpu_full.sh'
# test FAILURES (pytest exit 1) do not stop the later steps; a timeout, abort or crash does
OUT=gpurun_out/${TAG:-r03d}; mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] exit $rc"; grep -E "^FAILED|passed|failed" $OUT/pytest_gpu.log | tail -15
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '"metric"' $OUT/bench.log | cut -c1-400
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --steps 5 --warmup 2 --no-mode-r --no-fp16 --no-extras --no-op-timing --cpu-baseline off > $R/$OUT/prof.log 2>&1 || { tail -20 $R/$OUT/prof.log; exit 1; }
cd $R; f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 $f | head -25
