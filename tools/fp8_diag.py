"""Diagnostics for dclip_attn_fwd_fp8: compare the packed e4m3 planes with torch's float8_e4m3fn
conversion of the same scaled values (rounding mode, subnormals), byte by byte."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseclip_vit_multimodal_amd import _native as N
from denseclip_vit_multimodal_amd import ops

torch.manual_seed(0)
B, Nt, H = 1, 64, 1
C = 64 * H
qkv = torch.randn(B * Nt, 3 * C, device="cuda")
# column 0 of q / k / v: a ladder of magnitudes down into the e4m3 subnormal range after scaling
ladder = torch.tensor([448.0 * 2.0 ** (-e / 4.0) for e in range(64)], device="cuda")
qkv[:, 0] = ladder
qkv[:, C] = ladder * 0.37
qkv[:, 2 * C] = ladder * 1.3
qkv = qkv.to(torch.bfloat16)
ws = torch.zeros(N.lib().dclip_attn_fwd_fp8_workspace(B, Nt, H), dtype=torch.uint8, device="cuda")
o = torch.empty(B * Nt, C, dtype=torch.bfloat16, device="cuda")
lse = torch.empty(B * H * Nt, dtype=torch.float32, device="cuda")
N.call("dclip_attn_fwd_fp8", N.BF16, ops._p(qkv), ops._p(o), ops._p(lse), ops._p(ws), B, Nt, H, 64, ops._stream())
torch.cuda.synchronize()
npad = 64
plane = B * H * npad * 64
q8 = ws[:plane].view(Nt, 64)
k8 = ws[plane:2 * plane].view(Nt, 64)
amax = ws[3 * plane:3 * plane + 12].view(torch.float32)
print("amax hw", amax.tolist())
x = qkv.float()
for name, hw, cols in (("q", q8, slice(0, C)), ("k", k8, slice(C, 2 * C))):
    a = x[:, cols].abs().max()
    ref = (x[:, cols] * (448.0 / a)).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    mism = (ref != hw)
    print(name, "amax", float(a), "mismatching bytes", int(mism.sum()), "of", mism.numel())
    idx = mism.nonzero()[:12]
    for r, c in idx.tolist():
        v = float(x[r, cols][c] * (448.0 / a))
        print(f"   val {v:.6g}  hw {int(hw[r, c]):#04x} ({float(hw[r, c:c+1].view(torch.float8_e4m3fn).float()):.6g})"
              f"  torch {int(ref[r, c]):#04x} ({float(ref[r, c:c+1].view(torch.float8_e4m3fn).float()):.6g})")
    col0 = [(float(x[r, cols][0] * (448.0 / a)), int(hw[r, 0]), int(ref[r, 0])) for r in range(0, 64, 4)]
    print("  ladder col0 (val, hw, torch):", [(f"{v:.3g}", hex(h), hex(t)) for v, h, t in col0])

# ---- part 2: N = 1 (lse = the single score): kernel S vs q8 . k8 of the kernel's own planes
import math  # noqa: E402
for dt, code in ((torch.bfloat16, N.BF16), (torch.float16, N.F16)):
    torch.manual_seed(0)
    B, Nt, H = 2, 1, 3
    C = 64 * H
    qkv = (torch.randn(B * Nt, 3 * C, device="cuda") * 1.5).to(dt)
    qkv[:, :C] = (qkv[:, :C].float() * (64 ** -0.5 * 1.4426950408889634)).to(dt)
    ws = torch.zeros(N.lib().dclip_attn_fwd_fp8_workspace(B, Nt, H), dtype=torch.uint8, device="cuda")
    o = torch.empty(B * Nt, C, dtype=dt, device="cuda")
    lse = torch.empty(B * H * Nt, dtype=torch.float32, device="cuda")
    N.call("dclip_attn_fwd_fp8", code, ops._p(qkv), ops._p(o), ops._p(lse), ops._p(ws), B, Nt, H, 64, ops._stream())
    torch.cuda.synchronize()
    plane = B * H * 64 * 64
    q8 = ws[:plane].view(B, H, 64, 64)[:, :, 0].contiguous().view(torch.float8_e4m3fn).double()
    k8 = ws[plane:2 * plane].view(B, H, 64, 64)[:, :, 0].contiguous().view(torch.float8_e4m3fn).double()
    amax = ws[3 * plane:3 * plane + B * 3 * H * 4].view(torch.float32).view(B, 3, H).double()
    x = qkv.double().view(B, 3, H, 64)
    print(dt, "amax hw", amax.flatten().tolist())
    print(dt, "amax torch", x.abs().amax(-1).flatten().tolist())
    s_planes = (q8 * k8).sum(-1) * (amax[:, 0] / 448) * (amax[:, 1] / 448)
    print(dt, "lse (kernel S)", lse.view(B, H).tolist())
    print(dt, "S from planes ", s_planes.tolist())
    ref8q = (x[:, 0] * (448 / amax[:, 0:1].transpose(1, 2))).clamp(-448, 448)
    print(dt, "plane q8 == torch e4m3 of the scaled q:",
          bool(((ref8q.float().to(torch.float8_e4m3fn).double()) == q8).all()))
