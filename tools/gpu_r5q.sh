# attention passes with streaming output stores (ab/nts) vs base: per-pass rocprof means, fwd + bwd
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5q; mkdir -p $O
for v in ${VARIANTS:-base nts base nts}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v -o run -- python3 tools/attn_pass_probe.py ab/$v/libdclip.so 12 fwd > $O/$v.log 2>&1 || exit 3
  f=$(find $O/p_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "attn_bwd_dq2|attn_bwd_dkdv6|attn_fwd3|row0" $f | awk -F, '{printf "%s %s calls, avg %.1f us\n", substr($1,1,40), $2, $4/1000}'
  rm -rf $O/p_$v
done
