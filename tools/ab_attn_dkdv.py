"""A/B of the dK/dV pass variants at the headline shape (B = 8, N = 8193, H = 12) in ONE process:
the whole attention backward (dQ pass + dK/dV pass + fold merge) under DCLIP_OPT_ATTN_BWD_BLOCK 6
(dkdv6) and 7 (the software-pipelined dkdv7), arms alternated (ABBA) over rounds; per-launch mean
and min from HIP events on the launch stream; outputs compared bit for bit.

  python tools/ab_attn_dkdv.py [--rounds 6 --reps 10 --dtype bf16]
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
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--arms", default="6,7")
    a = ap.parse_args()
    from denseclip_vit_multimodal_amd import ops, _native as N_
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    B, N, H = 8, 8193, 12
    C = 64 * H
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * N, 3 * C, device="cuda", generator=g).to(dt)
    qkv[:, :C] = (qkv[:, :C].float() * (64 ** -0.5 * 1.4426950408889634)).to(dt)
    dout = torch.randn(B * N, C, device="cuda", generator=g).to(dt)
    o, lse = ops.attn_fwd(qkv, B, N, H, 64 ** -0.5)
    arms = [int(x) for x in a.arms.split(",")]
    outs = {}
    for v in arms:
        N_.call("dclip_set_option", N_.OPT_ATTN_BWD_BLOCK, v)
        outs[v] = ops.attn_bwd(qkv, o, dout, lse, B, N, H, 64 ** -0.5)
    torch.cuda.synchronize()
    t = {v: [] for v in arms}
    for r in range(a.rounds):
        order = arms if r % 2 == 0 else arms[::-1]
        for v in order:
            N_.call("dclip_set_option", N_.OPT_ATTN_BWD_BLOCK, v)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            ev[0].record()
            for i in range(a.reps):
                ops.attn_bwd(qkv, o, dout, lse, B, N, H, 64 ** -0.5)
                ev[i + 1].record()
            torch.cuda.synchronize()
            t[v] += [ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps)]
    N_.call("dclip_set_option", N_.OPT_ATTN_BWD_BLOCK, 0)
    flops = 10.0 * B * H * N * N * 64
    res = {f"block{v}": {"ms_mean": round(sum(x) / len(x), 4), "ms_min": round(min(x), 4),
                         "frac": round(flops / (sum(x) / len(x)) / 1e9 / 2500.0, 4)} for v, x in t.items()}
    res["bitwise_equal"] = all(torch.equal(outs[arms[0]], outs[v]) for v in arms[1:])
    res["dtype"] = a.dtype
    print(json.dumps(res))


if __name__ == "__main__":
    main()
