"""Run-to-run determinism of one train-step backward at the bench's widths (ViT-B/16 DenseCLIP,
mode F, B = 2 @ 512x1024): two fresh models from one seed, the same batch, forward + loss +
backward; reports whether the loss and every gradient are bit-identical, per compute dtype
(bf16 images; fp16 = fp32 images with the fp16 backbone), and the worst relative difference.

  python tools/determinism_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def one(cdt):
    from denseclip_vit_multimodal_amd import train
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = bench.make_model(dev, "F").train()
    m.backbone.compute_dtype = cdt
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    img_dt = torch.float32 if cdt == torch.float16 else torch.bfloat16
    img, seg, depth, mask = train.synth_batch(2, 512, 1024, dev, 0, image_dtype=img_dt)
    out = m(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True)
    loss = train.loss_fn(out, seg, depth, mask)
    loss.backward()
    torch.cuda.synchronize()
    return float(loss), {n: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None}


def main():
    for name, cdt in (("bf16", torch.bfloat16), ("fp16", torch.float16)):
        la, ga = one(cdt)
        lb, gb = one(cdt)
        diff = []
        for n in ga:
            if not torch.equal(ga[n], gb[n]):
                diff.append((float((ga[n] - gb[n]).abs().max()) / (float(ga[n].abs().max()) + 1e-30), n))
        diff.sort(reverse=True)
        print(f"{name}: loss {la!r} vs {lb!r} (equal {la == lb}); {len(ga)} gradients, {len(diff)} not bit-identical",
              flush=True)
        for d, n in diff[:12]:
            print(f"    {d:.3e}  {n}")


if __name__ == "__main__":
    main()
