"""A/B of the attention backward at the headline shape (B = 8, N = 8193, H = 12, bf16) in ONE
process: dclip_attn_bwd (16-bit dQ + dK/dV passes) against dclip_attn_bwd_fp8 (configs[4]: the
dK/dV pass on the block-scaled e4m3 MFMA), both on the fp8 forward's (o, lse), arms alternated
(ABBA) over rounds; per-launch mean and min from HIP events on the launch stream.

  python tools/ab_attn_bwd_fp8.py [--rounds 6 --reps 10]
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
    a = ap.parse_args()
    from denseclip_vit_multimodal_amd import ops
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    B, N, H = a.B, a.N, 12
    C = 64 * H
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * N, 3 * C, device="cuda", generator=g).to(dt)
    qkv[:, :C] = (qkv[:, :C].float() * (64 ** -0.5 * 1.4426950408889634)).to(dt)
    dout = torch.randn(B * N, C, device="cuda", generator=g).to(dt)
    o, lse = ops.attn_fwd_fp8(qkv, B, N, H)
    arms = {"bf16": False, "fp8": True}
    for f in arms.values():
        ops.attn_bwd(qkv, o, dout, lse, B, N, H, 64 ** -0.5, fp8=f)
    torch.cuda.synchronize()
    t = {k: [] for k in arms}
    for r in range(a.rounds):
        order = list(arms) if r % 2 == 0 else list(arms)[::-1]
        for name in order:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            ev[0].record()
            for i in range(a.reps):
                ops.attn_bwd(qkv, o, dout, lse, B, N, H, 64 ** -0.5, fp8=arms[name])
                ev[i + 1].record()
            torch.cuda.synchronize()
            t[name] += [ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps)]
    flops = 10.0 * B * H * N * N * 64
    res = {}
    for k, v in t.items():
        m = sum(v) / len(v)
        res[k] = {"ms_mean": round(m, 4), "ms_min": round(min(v), 4), "useful_tflops": round(flops / m / 1e9, 1)}
    res["fp8_over_bf16_time"] = round(res["fp8"]["ms_mean"] / res["bf16"]["ms_mean"], 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
