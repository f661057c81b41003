OUT=gpurun_out/r6aq; mkdir -p $OUT; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "dq_reduce_lds or test_attention_onepass_bwd" -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/ab_dq_reduce.py > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o ab -- python3 $R/tools/ab_dq_reduce.py --rounds 2 --reps 5 > $R/$OUT/prof.log 2>&1 || { tail $R/$OUT/prof.log; exit 1; }
cd $R; f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -8
