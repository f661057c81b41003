"""Per-row error of dclip_attn_fwd_fp8 against the float64 emulation (tests/test_gpu_fp8.py)."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from test_gpu_fp8 import make_qkv, emulate, pick, exact  # noqa: E402
from denseclip_vit_multimodal_amd import ops  # noqa: E402

for dt in (torch.bfloat16, torch.float16):
    torch.manual_seed(0)
    B, N, H = 2, 2049, 3
    qkv = make_qkv(B, N, H, dt)
    o, lse = ops.attn_fwd_fp8(qkv, B, N, H)
    o, lse = pick(o, lse, B, N, H, torch.arange(N))
    ref, lref = emulate(qkv, B, N, H)
    ex = exact(qkv, B, N, H)
    err = ((o - ref).norm(dim=-1) / ref.norm(dim=-1))  # (B, N)
    top = err.flatten().topk(8)
    print(dt, "total", float((o - ref).norm() / ref.norm()), "median row", float(err.median()))
    for v, i in zip(top.values.tolist(), top.indices.tolist()):
        b, r = divmod(i, N)
        print(f"   b {b} row {r} err {v:.4f} |ref| {float(ref[b, r].norm()):.4f} |exact| {float(ex[b, r].norm()):.4f}"
              f" lse {float(lse[b, :, r].max()):.3f}/{float(lref[b, :, r].max()):.3f}")
    perhead = [float((o[..., 64 * h:64 * h + 64] - ref[..., 64 * h:64 * h + 64]).norm() /
                     ref[..., 64 * h:64 * h + 64].norm()) for h in range(H)]
    print("   per head", perhead)
