#!/bin/bash
# one-pass backward option check: the bitwise tests, the ABBA A/B and a rocprofv3 kernel-stats run of it
#   gpurun -- 'TAG=r6av OPT=ATTN_PREP_ORDER bash tools/gpu_ab_bwd1_opt.sh'
OUT=gpurun_out/${TAG:-r6av}; mkdir -p $OUT; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "dq_reduce_lds" -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_dq_reduce.py --opt $OPT > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o ab -- python3 $R/tools/ab_dq_reduce.py --opt $OPT --rounds 2 --reps 5 > $R/$OUT/prof.log 2>&1 || { tail $R/$OUT/prof.log; exit 1; }
cd $R; f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -8
