"""Bias-gradient column-sum cost inside weight_grad at the bench shapes: time with want_bias
minus time without (same TN GEMM), per dY width.  DCLIP_LIB selects the library build.

  DCLIP_LIB=... python tools/colsum_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402

M = 8 * 8193
torch.manual_seed(0)


def ev(fn, reps=10):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


tot = 0.0
for n, k in [(3072, 768), (768, 3072), (768, 768), (2304, 768)]:
    dy = torch.randn(M, n, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, k, device="cuda").to(torch.bfloat16)
    w = [ev(lambda: O.weight_grad(dy, x, want_bias=True)) for _ in range(3)]
    wo = [ev(lambda: O.weight_grad(dy, x, want_bias=False)) for _ in range(3)]
    d = sorted(w)[1] - sorted(wo)[1]
    tot += d
    print(f"dY width {n:5d}: colsum adds {d * 1e3:7.1f} us ({M * n * 2 / (d * 1e-3) / 1e12 if d > 0 else 0:.2f} TB/s)")
print(f"per block backward: {tot * 1e3:.1f} us")
