"""A short target for rocprofv3 kernel traces of the train step (mode F, B = 8 @ 1024x2048):
W untimed + K steps, bf16 images or (--fp16) fp32 images with the fp16 compute dtype.

  python tools/step_runner.py [--fp16] [--warmup 3] [--steps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fp16", action="store_true")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    from denseclip_vit_multimodal_amd.train import synth_batch, make_optimizer
    dev = torch.device("cuda", 0)
    model = bench.make_model(dev, "F")
    if a.fp16:
        model.backbone.compute_dtype = torch.float16
    model.train()
    opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
    batch = synth_batch(8, 1024, 2048, dev, 0, image_dtype=torch.float32 if a.fp16 else torch.bfloat16)
    silog = SILogLoss()
    bench.run_steps(model, opt, batch, a.warmup, silog)
    torch.cuda.synchronize()
    bench.run_steps(model, opt, batch, a.steps, silog)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
