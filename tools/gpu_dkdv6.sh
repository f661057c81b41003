#!/bin/bash
# dK/dV pass variant 6 (64 keys per wave, AGPR dK / dV): correctness vs the default pass, timing, kernel trace
OUT=gpurun_out/${TAG:-r03b}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/ab_attn_opt.py 8 0 6 > $OUT/ab_bf16.log 2>&1; rc=$?; cat $OUT/ab_bf16.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/ab_attn_opt.py 8 0 6 --dt f16 > $OUT/ab_f16.log 2>&1; rc=$?; cat $OUT/ab_f16.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/ab_attn_opt.py 8 0 6 --n 10659 --h 16 --b 2 > $OUT/ab_vitl.log 2>&1; rc=$?; cat $OUT/ab_vitl.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && DCLIP_OPTIONS=8=6 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o k -- python3 $GRAFT_REPO_ROOT/tools/ab_attn_opt.py 8 6 --rounds 2 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT; find $OUT/prof -name "*stats*" | head; f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 $f | head -12; exit $rc
