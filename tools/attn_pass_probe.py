"""Run the headline-shape attention backward (B 8 x H 12 x N 8193, bf16) from one libdclip.so build,
for per-pass kernel times under rocprofv3 --stats (one build per process):

  rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o run -- python3 tools/attn_pass_probe.py ab/X/libdclip.so [reps] [fwd]
(fwd: the forward `reps` times too)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import _native  # noqa: E402

B, NT, C, H = 8, 8193, 768, 12
L = _native.load(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
DT, TDT = 2, torch.bfloat16
torch.manual_seed(0)
qkv = torch.randn(B * NT, 3 * C, device="cuda").to(TDT)
dout = torch.randn(B * NT, C, device="cuda").to(TDT)
o = torch.empty(B * NT, C, device="cuda", dtype=TDT)
lse = torch.empty(B * H * NT, device="cuda")
delta = torch.empty(L.dclip_attn_bwd_workspace(B, NT, H), device="cuda")
dqkv = torch.empty_like(qkv)
st = torch.cuda.current_stream().cuda_stream
for _ in range(reps if len(sys.argv) > 3 and sys.argv[3] == "fwd" else 1):
    assert L.dclip_attn_fwd(DT, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, NT, H, 64, 0.125, st) == 0
for _ in range(reps):
    assert L.dclip_attn_bwd(DT, qkv.data_ptr(), o.data_ptr(), dout.data_ptr(), lse.data_ptr(), delta.data_ptr(),
                            dqkv.data_ptr(), B, NT, H, 64, 0.125, st) == 0
torch.cuda.synchronize()
print("done", sys.argv[1])
