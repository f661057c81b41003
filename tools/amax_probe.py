"""Times the fp16 backward's gradient-scale kernels at the bench shape (8 x 8193 tokens x 768):
dclip_grad_scale over an fp32 gradient, dclip_add_readout_amax (read-out fold + scale in one pass)
and the torch ops it replaced (16->32-bit copy, CLS zeroing, unscale, add, then grad_scale).

  python tools/amax_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops  # noqa: E402


def ev(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


B, N, C = 8, 8193, 768
dev = torch.device("cuda", 0)
a = torch.randn(B * N, C, device=dev) * 1e-6
b = (torch.randn(B * N, C, device=dev) * 8).half()
hs = torch.tensor([2.0 ** 20, 2.0 ** -20, 0.0, 0.0], device=dev)


def old():
    dr = b.float()
    dr.view(B, N, C)[:, 0].zero_()
    s = a + dr.mul_(hs[1])
    return ops.grad_scale(s, torch.float16)


res = {"grad_scale (201 MB f32)": ev(lambda: ops.grad_scale(a, torch.float16)),
       "add_readout_amax (fused)": ev(lambda: ops.D().add_readout_amax(a, b, N, hs, ops.FP16_GRAD_AMAX)),
       "torch copy + zero + unscale + add + grad_scale": ev(old)}
for k, v in res.items():
    print(f"{k:50s} {v:8.1f} us")
