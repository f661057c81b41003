"""A/B kernel-variant options of the attention passes in ONE process (interleaved rounds, same
device, same random data): dclip_set_option(OPT, value) for each value, the headline shape.

  python tools/ab_attn_opt.py OPT_ID v0 v1 [...] [--dt bf16|f16] [--n N] [--rounds R]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import _native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("opt", type=int)
ap.add_argument("values", type=int, nargs="+")
ap.add_argument("--dt", default="bf16")
ap.add_argument("--n", type=int, default=8193)
ap.add_argument("--b", type=int, default=8)
ap.add_argument("--h", type=int, default=12)
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--fwd", action="store_true", help="time the forward instead of the backward")
a = ap.parse_args()
B, NT, H = a.b, a.n, a.h
C = 64 * H
L = _native.load()
dt = torch.bfloat16 if a.dt == "bf16" else torch.float16
code = 2 if a.dt == "bf16" else 1
torch.manual_seed(0)
qkv = torch.randn(B * NT, 3 * C, device="cuda").to(dt)
qkv[:, :C] *= 0.125 * 1.4426950408889634
dout = torch.randn(B * NT, C, device="cuda").to(dt)
o = torch.empty(B * NT, C, device="cuda", dtype=dt)
lse = torch.empty(B * H * NT, device="cuda")
delta = torch.empty(L.dclip_attn_bwd_workspace(B, NT, H), device="cuda")
dqkv = torch.empty_like(qkv)
st = torch.cuda.current_stream().cuda_stream
assert L.dclip_attn_fwd(code, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, NT, H, 64, 0.125, st) == 0


def bwd():
    assert L.dclip_attn_bwd(code, qkv.data_ptr(), o.data_ptr(), dout.data_ptr(), lse.data_ptr(), delta.data_ptr(),
                            dqkv.data_ptr(), B, NT, H, 64, 0.125, st) == 0


def fwd():
    assert L.dclip_attn_fwd(code, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, NT, H, 64, 0.125, st) == 0


def ev(fn, reps=3):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


outs = []
for v in a.values:
    L.dclip_set_option(a.opt, v)
    if a.fwd:
        o.zero_()
        fwd()
        torch.cuda.synchronize()
        outs.append(o.clone())
        continue
    dqkv.zero_()
    bwd()
    torch.cuda.synchronize()
    outs.append(dqkv.clone())
ref = outs[0].float()
for v, d in zip(a.values[1:], outs[1:]):
    df = (d.float() - ref)
    print(f"opt {a.opt}={v} vs {a.values[0]}: equal {torch.equal(d, outs[0])}, max|d| {float(df.abs().max()):.3e}, "
          f"rel {float(df.norm() / ref.norm()):.3e}, finite {bool(torch.isfinite(d).all())}", flush=True)
t = {v: [] for v in a.values}
for r in range(a.rounds):
    for v in a.values:
        L.dclip_set_option(a.opt, v)
        t[v].append(ev(fwd if a.fwd else bwd))
L.dclip_set_option(a.opt, 0)
fl = (4.0 if a.fwd else 10.0) * B * H * NT * NT * 64
for v in a.values:
    s = sorted(t[v])
    print(f"opt {a.opt}={v}: {'fwd' if a.fwd else 'bwd'} med {s[len(s) // 2]:.3f} min {s[0]:.3f} ms  ({fl / (s[len(s) // 2] * 1e-3) / 1e12:.0f} "
          f"TFLOP/s useful)", flush=True)
