"""What the fused bias-gradient column sums cost the weight-gradient GEMM: ops.weight_grad on the
ViT-B/16 block's four shapes at the headline batch, with the bias gradient (fused column sums,
the default), with it as a separate pass (DCLIP_OPT_GEMM_TN_COLSUM 1) and without it
(want_bias=False: the GEMM alone).  Interleaved rounds, median of 5.

  python tools/ab_wgrad_colsum.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import _native as N  # noqa: E402
from denseclip_vit_multimodal_amd import ops  # noqa: E402

M = 8 * 8193
shapes = {"in_proj": (2304, 768), "out_proj": (768, 768), "c_fc": (3072, 768), "c_proj": (768, 3072)}
torch.manual_seed(0)
data = {k: (torch.randn(M, n, device="cuda").to(torch.bfloat16), torch.randn(M, kk, device="cuda").to(torch.bfloat16))
        for k, (n, kk) in shapes.items()}


def ev(fn, reps=5):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


tot = {"fused colsum": 0.0, "separate colsum": 0.0, "no bias grad": 0.0}
for k, (dy, x) in data.items():
    t = {n: [] for n in tot}
    for r in range(5):
        N.call("dclip_set_option", N.OPT_GEMM_TN_COLSUM, 0)
        t["fused colsum"].append(ev(lambda: ops.weight_grad(dy, x)))
        N.call("dclip_set_option", N.OPT_GEMM_TN_COLSUM, 1)
        t["separate colsum"].append(ev(lambda: ops.weight_grad(dy, x)))
        N.call("dclip_set_option", N.OPT_GEMM_TN_COLSUM, 0)
        t["no bias grad"].append(ev(lambda: ops.weight_grad(dy, x, want_bias=False)))
    fl = 2.0 * M * dy.shape[1] * x.shape[1]
    for n in tot:
        v = sorted(t[n])[2]
        tot[n] += v
    print(k, "  ".join(f"{n}: {sorted(t[n])[2]:.3f} ms {fl / sorted(t[n])[2] / 1e9:.0f} TF/s" for n in tot), flush=True)
print("block total", "  ".join(f"{n}: {v:.3f} ms" for n, v in tot.items()))
