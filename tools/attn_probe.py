"""Run the fused attention forward and backward at the benchmark shape (B=8, N=8193, H=12,
bf16) a few times — a short target for rocprofv3 --pmc passes.

  python tools/attn_probe.py [reps] [values of DCLIP_OPT_ATTN_BWD_BLOCK, e.g. 0,1,2]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import _native  # noqa: E402
from denseclip_vit_multimodal_amd import ops as O  # noqa: E402

B, NT, C, H = 8, 8193, 768, 12
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
variants = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [None]
qkv = torch.randn(B * NT, 3 * C, device="cuda").to(torch.bfloat16)
dout = torch.randn(B * NT, C, device="cuda").to(torch.bfloat16)
for v in variants:
    if v is not None:
        _native.call("dclip_set_option", _native.OPT_ATTN_BWD_BLOCK, v)
    for _ in range(reps):
        o, lse = O.attn_fwd(qkv, B, NT, H, 0.125)
        O.attn_bwd(qkv, o, dout, lse, B, NT, H, 0.125)
torch.cuda.synchronize()
print("done")
