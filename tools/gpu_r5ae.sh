# where GradAllReduce's world-size-1 cost sits: hooks only / all-reduce after the backward / full
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5ae; mkdir -p $O
for v in none hooksonly nohooks allreduce allreduce nohooks hooksonly none; do
  MASTER_PORT=$((29600 + RANDOM % 200)) timeout -k 10 200 python3 tools/ddp_probe.py $v 10 >> $O/ddp_probe.log 2>&1 || { tail -20 $O/ddp_probe.log; exit 3; }
done
grep "ms/step" $O/ddp_probe.log | grep -v print
