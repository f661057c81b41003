#!/bin/bash
# one gpurun call of checks + A/Bs:  gpurun --timeout 1500 -- 'TAG=r03g PYARGS="..." AB="..." CONFIGS=1 bash tools/gpu_round.sh'
#   PYARGS  pytest files / options (run first; test failures do not stop the call, a timeout / crash does)
#   PYK     pytest -k expression (spaces allowed)
#   AB      a command line run next (e.g. "python -u tools/ab_wgrad_opt.py 0 4")
#   CONFIGS 1: then tools/gpu_configs.sh (MFMA ceiling probe + the BASELINE config lines)
OUT=gpurun_out/${TAG:-r03}; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$PYARGS" ]; then
  if [ -n "$PYK" ]; then KARG=(-k "$PYK"); else KARG=(); fi
  timeout -k 10 600 python -u -m pytest $PYARGS "${KARG[@]}" -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "[pytest] exit $rc"; grep -E "^FAILED|passed|failed" $OUT/pytest.log | tail -12
  [ $rc -gt 1 ] && exit $rc
fi
if [ -n "$AB" ]; then
  timeout -k 10 300 $AB > $OUT/ab.log 2>&1; rc=$?; echo "[ab] exit $rc"; tail -20 $OUT/ab.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "$CONFIGS" = "1" ]; then TAG=$TAG bash tools/gpu_configs.sh || exit $?; fi
exit 0
