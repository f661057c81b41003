"""Byte-compare every packed plane of dclip_attn_fwd_fp8 (q8 / k8 rows, their E8M0 scales, the
de-permuted vt8 and the per-unit scale dwords) with a torch restatement of fp8mx_pack_kernel
(attention_fp8.hip), for the test shape B=2, N=2049, H=3 (tokens 1..N-1 in 64-token units).
Runs the all-e4m3 kernel (DCLIP_OPT_ATTN_FP8_QK 1): the default one packs V^T only.

  python tools/fp8_planes.py
"""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from test_gpu_fp8 import make_qkv, mx_quant, PERM  # noqa: E402
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402
from denseclip_vit_multimodal_amd import ops  # noqa: E402


def main():
    assert N.lib().dclip_set_option(N.OPT_ATTN_FP8_QK, 1) == 0
    ok_all = True
    for dt, code in ((torch.bfloat16, N.BF16), (torch.float16, N.F16)):
        torch.manual_seed(0)
        B, Nt, H = 2, 2049, 3
        n1 = Nt - 1
        n1p = (n1 + 63) // 64 * 64
        qkv = make_qkv(B, Nt, H, dt)
        ws = torch.zeros(N.lib().dclip_attn_fwd_fp8_workspace(B, Nt, H), dtype=torch.uint8, device="cuda")
        o = torch.empty(B * Nt, 64 * H, dtype=dt, device="cuda")
        lse = torch.empty(B * H * Nt, dtype=torch.float32, device="cuda")
        N.call("dclip_attn_fwd_fp8", code, ops._p(qkv), ops._p(o), ops._p(lse), ops._p(ws), B, Nt, H, 64, ops._stream())
        torch.cuda.synchronize()
        ws = ws.cpu()
        plane = B * H * n1p * 64
        q8 = ws[:plane].view(B, H, n1p, 64)
        k8 = ws[plane:2 * plane].view(B, H, n1p, 64)
        vt8 = ws[2 * plane:3 * plane].view(B, H, 64, n1p // 64, 64)
        qs = ws[3 * plane:3 * plane + B * H * n1p * 2].view(B, H, n1p, 2)
        o0 = 3 * plane + B * H * n1p * 2
        sc = ws[o0:o0 + B * H * (n1p // 64) * 256].view(B, H, n1p // 64, 2, 32, 4)  # [unit][half][r][byte]
        x = torch.zeros(B, n1p, 3, H, 64, dtype=torch.float32)
        x[:, :n1] = qkv.float().cpu().view(B, Nt, 3, H, 64)[:, 1:]
        q, k, v = x.permute(2, 0, 3, 1, 4)  # (B, H, n1p, 64)
        rq, eq = mx_quant(q.reshape(B, H, n1p, 2, 32))
        rk, ek = mx_quant(k.reshape(B, H, n1p, 2, 32))
        # V^T: blocks of 32 keys (the unit's halves) per head dim d; slot s of a unit holds key PERM[s]
        U = n1p // 64
        vu = v.reshape(B, H, U, 2, 32, 64).permute(0, 1, 2, 5, 3, 4)  # (B, H, U, d, key half, 32)
        rv, ev = mx_quant(vu)
        rv = rv.reshape(B, H, U, 64, 64)[..., PERM].permute(0, 1, 3, 2, 4)  # (B, H, d, U, slot)
        checks = [
            ("q8", q8, rq.reshape(B, H, n1p, 64)), ("k8", k8, rk.reshape(B, H, n1p, 64)),
            ("vt8", vt8, rv),
            ("q scales", qs, (127 - eq).to(torch.uint8).reshape(B, H, n1p, 2)),
            # key kb * 32 + r of a unit, d-half `half` -> sc[unit][half][r][byte kb]
            ("K scales", sc[..., :2], (127 - ek).to(torch.uint8).reshape(B, H, n1p // 64, 2, 32, 2).permute(0, 1, 2, 5, 4, 3)),
            # head dim db * 32 + r, key half `half` -> sc[unit][half][r][byte 2 + db]
            ("V scales", sc[..., 2:], (127 - ev).to(torch.uint8).reshape(B, H, U, 2, 32, 2).permute(0, 1, 2, 5, 4, 3)),
        ]
        for name, hw, ref in checks:
            mism = int((hw != ref).sum())
            ok_all &= mism == 0
            print(dt, name, "mismatching", mism, "of", hw.numel(), flush=True)
    print("fp8 planes bit-exact:", ok_all)
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
