#!/bin/bash
# rocprof per-kernel summary of the attention backward A/B (tools/ab_attn_bwd1.py) at the headline shape
#   gpurun -- 'TAG=r6l ARMS=0,9 bash tools/gpu_prof_bwd1.sh'
OUT=gpurun_out/${TAG:-r6}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/ab_attn_bwd1.py --rounds 2 --reps 5 --arms ${ARMS:-0,9} > $GRAFT_REPO_ROOT/$OUT/prof_ab.log 2>&1
rc=$?; python3 $GRAFT_REPO_ROOT/tools/rocpd_stats.py $(find $GRAFT_REPO_ROOT/$OUT/prof -name "*.db" | head -1) --filter attn --csv $GRAFT_REPO_ROOT/$OUT/kernel_stats.csv | cut -c1-150
exit $rc
