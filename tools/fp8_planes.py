"""Byte-compare every packed plane of dclip_attn_fwd_fp8 (q8, k8, de-permuted vt8, amax) with a
torch fp32 restatement, for the test shape B=2, N=2049, H=3."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from test_gpu_fp8 import make_qkv  # noqa: E402
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402
from denseclip_vit_multimodal_amd import ops  # noqa: E402


def kappa(half, j):
    t, reg = j >> 4, j & 15
    return 32 * t + (reg & 3) + 8 * (reg >> 2) + 4 * half


perm = torch.tensor([kappa(s >> 5, s & 31) for s in range(64)])
for dt, code in ((torch.bfloat16, N.BF16), (torch.float16, N.F16)):
    torch.manual_seed(0)
    B, Nt, H = 2, 2049, 3
    npad = (Nt + 63) // 64 * 64
    qkv = make_qkv(B, Nt, H, dt)
    ws = torch.zeros(N.lib().dclip_attn_fwd_fp8_workspace(B, Nt, H), dtype=torch.uint8, device="cuda")
    o = torch.empty(B * Nt, 64 * H, dtype=dt, device="cuda")
    lse = torch.empty(B * H * Nt, dtype=torch.float32, device="cuda")
    N.call("dclip_attn_fwd_fp8", code, ops._p(qkv), ops._p(o), ops._p(lse), ops._p(ws), B, Nt, H, 64, ops._stream())
    torch.cuda.synchronize()
    plane = B * H * npad * 64
    hw_amax = ws[3 * plane:3 * plane + B * 3 * H * 4].view(torch.float32).view(B, 3, H).cpu()
    x = qkv.float().cpu().view(B, Nt, 3, H, 64)
    amax = x.abs().amax(dim=(1, 4))
    print(dt, "amax equal", bool((amax == hw_amax).all()))
    sc = (torch.tensor(448.0) / amax)  # fp32 like the kernel
    ref = (x * sc.view(B, 1, 3, H, 1)).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    ref = ref.permute(2, 0, 3, 1, 4)  # (3, B, H, N, 64)
    q8 = ws[:plane].view(B, H, npad, 64).cpu()
    k8 = ws[plane:2 * plane].view(B, H, npad, 64).cpu()
    vt8 = ws[2 * plane:3 * plane].view(B, H, 64, npad // 64, 64).cpu()
    # vt8[b][h][d][u][slot] = v[u*64 + perm[slot]][d]
    v_from = torch.empty(B, H, npad // 64, 64, 64, dtype=torch.uint8)
    v_from[:, :, :, perm, :] = vt8.permute(0, 1, 3, 4, 2)
    v_from = v_from.reshape(B, H, npad, 64)
    for name, hw, r in (("q", q8, ref[0]), ("k", k8, ref[1]), ("v", v_from, ref[2])):
        mism = hw[:, :, :Nt] != r
        print(dt, name, "mismatching", int(mism.sum()), "of", mism.numel(), "per (b,h)",
              mism.sum(dim=(2, 3)).tolist(), "pad rows nonzero", int((hw[:, :, Nt:] != 0).sum()))
        if mism.any():
            b, h, t, d = mism.nonzero()[0].tolist()
            print("   first", (b, h, t, d), "val", float(x[b, t, "qkv".index(name), h, d] * sc[b, "qkv".index(name), h]),
                  "hw", int(hw[b, h, t, d]), "ref", int(r[b, h, t, d]))
