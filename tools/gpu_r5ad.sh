# GradAllReduce (wrap_ddp default) vs torch DDP vs none at world size 1 (RCCL): one process each, ABBA; DDP tests
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5ad; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_headline.py -k "ddp" tests/test_gpu_dropin_heads.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest.log | tail -5
[ $rc -le 1 ] || exit $rc
for v in none allreduce default default allreduce none; do
  MASTER_PORT=$((29600 + RANDOM % 200)) timeout -k 10 200 python3 tools/ddp_probe.py $v 10 >> $O/ddp_probe.log 2>&1 || { tail -20 $O/ddp_probe.log; exit 3; }
done
grep "ms/step" $O/ddp_probe.log | grep -v print
