"""Time the fp32 -> bf16 transposed weight copies (ViT-B/16 block shapes) on the current stream."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402

for shape in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
    x = torch.randn(*shape, device="cuda")
    for _ in range(5):
        O.transpose2d(x, torch.bfloat16)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 200
    e0.record()
    for _ in range(n):
        O.transpose2d(x, torch.bfloat16)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    print("transpose %s: %.2f us/launch  %.2f TB/s" % (shape, us, x.numel() * 6 / us / 1e6))
