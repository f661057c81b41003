"""A/B the attention kernel variants (dclip_set_option knobs) in ONE process at the bench
shape (B=8, N=8193, H=12, bf16, random data), interleaved rounds; checks that every
variant's outputs are bitwise identical to the default's.

  python tools/attn_variants.py [rounds]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402

B, NT, C, H = 8, 8193, 768, 12
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
# variants: "fwd_waves,dq_waves,dkdv_waves[,dkdv_qs[,bwd_kernel]]" strings after the round count
torch.manual_seed(0)
qkv = torch.randn(B * NT, 3 * C, device="cuda").to(torch.bfloat16)
dout = torch.randn(B * NT, C, device="cuda").to(torch.bfloat16)
FL = 4.0 * B * H * NT * NT * 64


def ev_time(fn, reps=3):
    fn()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def setopt(fw, dq, dkdv, qs=0, bk=0):
    N.call("dclip_set_option", N.OPT_ATTN_BWD_KERNEL, bk)  # 0 CLS-split passes, 1 generic
    N.call("dclip_set_option", N.OPT_ATTN_DKDV_QS, qs)
    N.call("dclip_set_option", N.OPT_ATTN_FWD_WAVES, fw)
    N.call("dclip_set_option", N.OPT_ATTN_DQ_WAVES, dq)
    N.call("dclip_set_option", N.OPT_ATTN_DKDV_WAVES, dkdv)


setopt(0, 0, 0)
o_ref, lse_ref = O.attn_fwd(qkv, B, NT, H, 0.125)
d_ref = O.attn_bwd(qkv, o_ref, dout, lse_ref, B, NT, H, 0.125)
variants = [tuple(int(x) for x in v.split(',')) for v in (sys.argv[2:] or ['8,4,4', '4,4,4', '8,8,8'])]
res = {v: {"fwd": [], "bwd": []} for v in variants}
for v in variants:
    setopt(*v)
    o, lse = O.attn_fwd(qkv, B, NT, H, 0.125)
    d = O.attn_bwd(qkv, o_ref, dout, lse_ref, B, NT, H, 0.125)
    same = (torch.equal(o, o_ref), torch.equal(lse, lse_ref), torch.equal(d, d_ref))
    print(f"variant fwd/dq/dkdv waves {v}: outputs bitwise equal to default: {same}", flush=True)
for r in range(rounds):
    for v in variants:
        setopt(*v)
        res[v]["fwd"].append(ev_time(lambda: O.attn_fwd(qkv, B, NT, H, 0.125)))
        res[v]["bwd"].append(ev_time(lambda: O.attn_bwd(qkv, o_ref, dout, lse_ref, B, NT, H, 0.125)))
for v in variants:
    f = sorted(res[v]["fwd"])[len(res[v]["fwd"]) // 2]
    b = sorted(res[v]["bwd"])[len(res[v]["bwd"]) // 2]
    print(f"{str(v):12s} fwd {f:7.3f} ms {FL / f / 1e9:7.1f} TF/s | bwd {b:7.3f} ms "
          f"{2.5 * FL / b / 1e9:7.1f} TF/s (5-matmul flops)", flush=True)
setopt(0, 0, 0)
