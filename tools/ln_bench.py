"""LayerNorm forward / backward at the bench shape (65544 x 768, f32 in, bf16 / f32 out) with
achieved HBM GB/s (algorithmic bytes: fwd reads x f32, writes y bf16; bwd reads dy f32, x f32,
dx f32 (accumulate) and writes dx f32)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402

R, C = 8 * 8193, 768
x = torch.randn(R, C, device="cuda")
w = torch.randn(C, device="cuda")
b = torch.randn(C, device="cuda")
dy = torch.randn(R, C, device="cuda")
dx = torch.randn(R, C, device="cuda")
dw = torch.zeros(C, device="cuda")
db = torch.zeros(C, device="cuda")
_, mu, rs = O.layernorm_fwd(x, w, b, torch.float32)


def ev(fn, reps=20):
    fn()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return a.elapsed_time(e) / reps


tf = ev(lambda: O.layernorm_fwd(x, w, b, torch.bfloat16))
tb = ev(lambda: O.layernorm_bwd(dy, x, w, mu, rs, dx, 1, dw, db))
print(f"ln fwd {tf * 1e3:.1f} us  {R * C * 6 / tf / 1e6:.0f} GB/s | ln bwd {tb * 1e3:.1f} us  "
      f"{R * C * 16 / tb / 1e6:.0f} GB/s")
