"""A/B the attention forward kernels in ONE process at the bench shape (B=8, N=8193, H=12,
bf16, random data), interleaved rounds: generic kernel vs the CLS-split kernel (4 / 8 waves).

  python tools/attn_fwd_ab.py [rounds]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402

B, NT, C, H = 8, 8193, 768, 12
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
torch.manual_seed(0)
qkv = torch.randn(B * NT, 3 * C, device="cuda").to(torch.bfloat16)
FL = 4.0 * B * H * NT * NT * 64
VARIANTS = {"generic8": (1, 8), "split8": (0, 8), "pipe8": (3, 0), "wide": (2, 0)}


def setv(k, w):
    N.call("dclip_set_option", N.OPT_ATTN_FWD_KERNEL, k)
    N.call("dclip_set_option", N.OPT_ATTN_FWD_WAVES, w)


def ev_time(fn, reps=5):
    fn()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


outs = {}
for name, v in VARIANTS.items():
    setv(*v)
    outs[name] = O.attn_fwd(qkv, B, NT, H, 0.125)
ref = outs["generic8"]
for name, (o, lse) in outs.items():
    d = (o.float() - ref[0].float()).abs().max().item()
    dl = (lse - ref[1]).abs().max().item()
    print(f"{name:10s} max|o - generic8| {d:.3e}  max|lse - generic8| {dl:.3e}", flush=True)
res = {k: [] for k in VARIANTS}
for r in range(rounds):
    for name, v in VARIANTS.items():
        setv(*v)
        res[name].append(ev_time(lambda: O.attn_fwd(qkv, B, NT, H, 0.125)))
for name in VARIANTS:
    t = sorted(res[name])
    print(f"{name:10s} median {t[rounds // 2]:.4f} ms  min {t[0]:.4f} ms  {FL / t[rounds // 2] / 1e9:.1f} TF/s",
          flush=True)
setv(0, 0)
