"""Timing of the diagnostic attention-forward variants (libdclip_diag.so, make -C csrc diag):
which part of the CLS-split forward is on the critical path.  Results of DIAG != 0 are
wrong by construction; only the times mean anything.

  DCLIP_LIB=denseclip_vit_multimodal_amd/libdclip_diag.so python tools/attn_diag.py [waves]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402

B, NT, C, H = 8, 8193, 768, 12
waves = int(sys.argv[1]) if len(sys.argv) > 1 else 8
torch.manual_seed(0)
qkv = torch.randn(B * NT, 3 * C, device="cuda").to(torch.bfloat16)
FL = 4.0 * B * H * NT * NT * 64
names = {0: "full", 11: "no barrier", 12: "no exp", 13: "no K/V staging", 14: "no PV mfma", 15: "no S mfma"}
N.call("dclip_set_option", N.OPT_ATTN_FWD_WAVES, waves)


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


res = {k: [] for k in names}
for r in range(5):
    for k in names:
        N.call("dclip_set_option", N.OPT_ATTN_FWD_KERNEL, k)
        res[k].append(ev_time(lambda: O.attn_fwd(qkv, B, NT, H, 0.125)))
for k, v in names.items():
    t = sorted(res[k])[2]
    print(f"{v:16s} {t:.4f} ms  ({FL / t / 1e9:.0f} TF/s-equivalent)", flush=True)
