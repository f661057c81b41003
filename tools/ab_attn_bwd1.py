"""A/B of the attention backward at the headline shape (B = 8, N = 8193, H = 12, bf16) in ONE
process: the two-pass backward (DCLIP_OPT_ATTN_BWD_BLOCK 0: dQ pass + dK/dV pass) against the
one-pass backward (option 9, attention_bwd1.hip: prep + one key-major sweep with per-key-block dQ
partials + the ordered dQ reduction), arms alternated (ABBA) over rounds; per-launch mean and min
from HIP events on the launch stream, and the two results compared (dK / dV bitwise, dQ norm-wise).

  python tools/ab_attn_bwd1.py [--rounds 6 --reps 10 --dtype bf16]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--N", type=int, default=8193)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--arms", default="0,9")
    a = ap.parse_args()
    from denseclip_vit_multimodal_amd import ops
    from denseclip_vit_multimodal_amd import _native as NT
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    B, N, H = a.B, a.N, 12
    C = 64 * H
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * N, 3 * C, device="cuda", generator=g).to(dt)
    qkv[:, :C] = (qkv[:, :C].float() * (64 ** -0.5 * 1.4426950408889634)).to(dt)
    dout = torch.randn(B * N, C, device="cuda", generator=g).to(dt)
    o, lse = ops.attn_fwd(qkv, B, N, H, 64 ** -0.5)
    arms = {f"opt{v}": int(v) for v in a.arms.split(",")}

    def run(v):
        NT.call("dclip_set_option", NT.OPT_ATTN_BWD_BLOCK, v)
        return ops.attn_bwd(qkv, o, dout, lse, B, N, H, 64 ** -0.5)

    outs = {k: run(v) for k, v in arms.items()}
    torch.cuda.synchronize()
    base = outs[list(arms)[0]].float()
    cmp = {}
    rest = torch.ones(B * N, dtype=torch.bool, device="cuda")
    rest[::N] = False
    for k, x in outs.items():
        x = x.float()
        cmp[k] = {"dkdv_bitwise": bool(torch.equal(x[rest, C:], base[rest, C:])),
                  "dq_rel": float((x[:, :C] - base[:, :C]).norm() / base[:, :C].norm()),
                  "dkdv_rel": float((x[:, C:] - base[:, C:]).norm() / base[:, C:].norm())}
    del outs
    t = {k: [] for k in arms}
    for r in range(a.rounds):
        order = list(arms) if r % 2 == 0 else list(arms)[::-1]
        for name in order:
            NT.call("dclip_set_option", NT.OPT_ATTN_BWD_BLOCK, arms[name])
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            ev[0].record()
            for i in range(a.reps):
                ops.attn_bwd(qkv, o, dout, lse, B, N, H, 64 ** -0.5)
                ev[i + 1].record()
            torch.cuda.synchronize()
            t[name] += [ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps)]
    NT.call("dclip_set_option", NT.OPT_ATTN_BWD_BLOCK, 0)
    flops = 10.0 * B * H * N * N * 64
    res = {"compare": cmp}
    for k, v in t.items():
        m = sum(v) / len(v)
        med = sorted(v)[len(v) // 2]
        res[k] = {"ms_mean": round(m, 4), "ms_median": round(med, 4), "ms_min": round(min(v), 4),
                  "ms_max": round(max(v), 4), "useful_tflops": round(flops / m / 1e9, 1),
                  "frac_of_2500": round(flops / m / 1e9 / 2500, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
