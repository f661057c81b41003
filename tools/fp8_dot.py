"""Accuracy of the fp8 MFMA dot product inside dclip_attn_fwd_fp8: with N = 1 the lse is the
single score S = sscale * sum_d q8[d] k8[d]; compare it with the exact float64 dot of the
kernel's own packed planes for heavy-tailed rows (a wide range of product magnitudes)."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402
from denseclip_vit_multimodal_amd import ops  # noqa: E402

torch.manual_seed(0)
for tail in (1, 3, 5):
    B, Nt, H = 64, 1, 1
    qkv = (torch.randn(B, 3 * 64, device="cuda") ** tail).to(torch.bfloat16)
    ws = torch.zeros(N.lib().dclip_attn_fwd_fp8_workspace(B, Nt, H), dtype=torch.uint8, device="cuda")
    o = torch.empty(B, 64, dtype=torch.bfloat16, device="cuda")
    lse = torch.empty(B, dtype=torch.float32, device="cuda")
    N.call("dclip_attn_fwd_fp8", N.BF16, ops._p(qkv), ops._p(o), ops._p(lse), ops._p(ws), B, Nt, H, 64, ops._stream())
    torch.cuda.synchronize()
    plane = B * 64 * 64
    q8 = ws[:plane].view(B, 64, 64)[:, 0].contiguous().view(torch.float8_e4m3fn).double().cpu()
    k8 = ws[plane:2 * plane].view(B, 64, 64)[:, 0].contiguous().view(torch.float8_e4m3fn).double().cpu()
    amax = ws[3 * plane:3 * plane + B * 12].view(torch.float32).view(B, 3).double().cpu()
    raw = (q8 * k8).sum(-1)
    exact = raw * (amax[:, 0] / 448) * (amax[:, 1] / 448)
    hw = lse.double().cpu()
    rawhw = hw / ((amax[:, 0] / 448) * (amax[:, 1] / 448))
    err = (rawhw - raw).abs()
    maxprod = (q8 * k8).abs().amax(-1)
    rel_to_max = err / maxprod
    print(f"tail {tail}: |S - S_exact| max {float((hw - exact).abs().max()):.3g}; raw-sum error / max|product|: "
          f"max {float(rel_to_max.max()):.3g} median {float(rel_to_max.median()):.3g}; "
          f"raw-sum error / |raw sum| max {float((err / raw.abs().clamp(min=1)).max()):.3g}")
