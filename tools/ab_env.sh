#!/bin/bash
# A/B an environment switch on the bench in alternating runs:  bash tools/ab_env.sh VAR "v1 v2" rounds tag
VAR=$1; VALS=$2; R=${3:-2}; TAG=${4:-ab}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-mode-r --cpu-baseline off > $OUT/b_$(echo $v | tr "/=" "__")_$r.log 2>&1 || exit $?
    echo "$VAR=$v round $r: $(grep -o "\"value\": [0-9.]*" $OUT/b_$(echo $v | tr "/=" "__")_$r.log)"
  done
done
