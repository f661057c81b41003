#!/bin/bash
# Round-6 gpurun body:  gpurun --timeout 1200 -- 'TAG=r6a PYARGS="tests -m gpu" BENCH="--steps 10" bash tools/gpu_r6.sh'
#   PYARGS  pytest selection (no -x: every failure is listed); a timeout / crash ends the call
#   PYK     pytest -k expression
#   BENCH   bench.py arguments (run when set, after pytest unless pytest crashed)
#   AB      a command run last (its own 300 s limit)
OUT=gpurun_out/${TAG:-r6}; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$PYARGS" ]; then
  if [ -n "$PYK" ]; then KARG=(-k "$PYK"); else KARG=(); fi
  timeout -k 10 720 python -u -m pytest $PYARGS "${KARG[@]}" -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "[pytest] exit $rc"; grep -E "^FAILED|passed|failed" $OUT/pytest.log | tail -15
  [ $rc -gt 1 ] && exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 480 python -u bench.py $BENCH > $OUT/bench.log 2>&1; rc=$?
  echo "[bench] exit $rc"; tail -c 3000 $OUT/bench.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$AB" ]; then
  timeout -k 10 300 $AB > $OUT/ab.log 2>&1; rc=$?; echo "[ab] exit $rc"; tail -30 $OUT/ab.log; [ $rc -ne 0 ] && exit $rc
fi
exit 0
