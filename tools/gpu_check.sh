#!/bin/bash
# One gpurun call: GPU tests, a short bench, and a rocprofv3 kernel-trace of the bench.
# Stops at the first step that faults, aborts or times out (exit status other than 0/1).
#   gpurun --timeout 1200 -- bash tools/gpu_check.sh [tag]
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp

ok() { # continue only after a clean exit or an ordinary test failure
  local rc=$1 step=$2
  echo "[$step] exit $rc" | tee -a $OUT/steps.log
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
}

if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; ok $? pytest
  tail -5 $OUT/pytest_gpu.log
fi
timeout -k 10 420 python bench.py --steps ${STEPS:-5} --warmup 2 > $OUT/bench.log 2>&1; ok $? bench
tail -c 3000 $OUT/bench.log
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 2 --no-mode-r --cpu-baseline off > $OUT/bench_prof.log 2>&1; ok $? rocprof
  find $OUT/prof -name '*kernel_stats.csv'
fi
