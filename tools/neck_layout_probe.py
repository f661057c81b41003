"""Probe: MIOpen time of the ViTFeatureFusionNeck + heads fwd+bwd, NCHW vs channels_last, bf16."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from denseclip_vit_multimodal_amd.models import ViTFeatureFusionNeck
from denseclip_vit_multimodal_amd.heads import FCNHead

dev = "cuda"
for fmt in (torch.contiguous_format, torch.channels_last):
    neck = ViTFeatureFusionNeck([768] * 12, 256, 128).to(dev).to(memory_format=fmt)
    head = FCNHead(256, 256).to(dev).to(memory_format=fmt)
    maps = [torch.randn(8, 768, 64, 128, device=dev, dtype=torch.bfloat16).contiguous(memory_format=fmt).requires_grad_(True)
            for _ in range(12)]
    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = head(neck(maps)[0])
        y.float().sum().backward()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    print(fmt, (time.perf_counter() - t) / 5 * 1e3, "ms / fwd+bwd")
