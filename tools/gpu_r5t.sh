# lean text blocks: step A/B (fp32 lean / plain / const) and the replay alone
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 600 python3 tools/text_probe.py 3 10 > $O/text_probe.log 2>&1 || exit 3
grep -v amdgpu.ids $O/text_probe.log | tail -12
