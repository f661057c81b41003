"""Run the fused attention forward and backward at the benchmark shape (B=8, N=8193, H=12,
bf16) a few times — a short target for rocprofv3 --pmc passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402

B, NT, C, H = 8, 8193, 768, 12
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
qkv = torch.randn(B * NT, 3 * C, device="cuda").to(torch.bfloat16)
dout = torch.randn(B * NT, C, device="cuda").to(torch.bfloat16)
for _ in range(reps):
    o, lse = O.attn_fwd(qkv, B, NT, H, 0.125)
    O.attn_bwd(qkv, o, dout, lse, B, NT, H, 0.125)
torch.cuda.synchronize()
print("done")
