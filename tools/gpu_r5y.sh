# whole train step replayed from one HIP graph (train.CapturedTrainStep) vs eager: ABBA A/B, bf16 and fp16
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5y; mkdir -p $O
timeout -k 10 500 python3 -u tools/graph_step_probe.py 4 10 > $O/graph_step.log 2>&1; rc=$?
grep -v amdgpu.ids $O/graph_step.log | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u tools/graph_step_probe.py 4 10 --fp16 > $O/graph_step_fp16.log 2>&1 || exit 4
grep -v amdgpu.ids $O/graph_step_fp16.log | tail -5
