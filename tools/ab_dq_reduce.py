"""A/B of a one-pass attention backward option, 0 vs 1 (--opt ATTN_DQ_REDUCE: the dQ reduction with 8
lanes per query vs 8 queries per workgroup read contiguously through LDS; --opt ATTN_PREP_ORDER: the
prep pass's workgroups query-block-major vs head-minor) at the headline shape (B = 8,
N = 8193, H = 12) in ONE process: bitwise comparison of the whole backward output, then the whole
backward timed per launch with HIP events on the launch stream, arms alternated (ABBA) over rounds.

  python tools/ab_dq_reduce.py [--opt ATTN_PREP_ORDER --rounds 8 --reps 10 --dtype bf16]
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
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--N", type=int, default=8193)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--opt", default="ATTN_DQ_REDUCE", help="the option name (OPT_<name> of _native): ATTN_DQ_REDUCE or ATTN_PREP_ORDER")
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
    arms = {"opt0": 0, "opt1": 1}
    OPT = getattr(NT, "OPT_" + a.opt)

    def run(v):
        NT.call("dclip_set_option", OPT, v)
        return ops.attn_bwd(qkv, o, dout, lse, B, N, H, 64 ** -0.5)

    outs = [run(v) for v in arms.values()]
    torch.cuda.synchronize()
    res = {"bitwise_equal": bool(torch.equal(outs[0], outs[1]))}
    del outs
    t = {k: [] for k in arms}
    for r in range(a.rounds):
        order = list(arms) if r % 2 == 0 else list(arms)[::-1]
        for name in order:
            NT.call("dclip_set_option", OPT, arms[name])
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            ev[0].record()
            for i in range(a.reps):
                ops.attn_bwd(qkv, o, dout, lse, B, N, H, 64 ** -0.5)
                ev[i + 1].record()
            torch.cuda.synchronize()
            t[name] += [ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps)]
    NT.call("dclip_set_option", OPT, 0)
    for k, v in t.items():
        s = sorted(v)
        res[k] = {"ms_mean": round(sum(v) / len(v), 4), "ms_median": round(s[len(s) // 2], 4),
                  "ms_min": round(s[0], 4), "ms_max": round(s[-1], 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
