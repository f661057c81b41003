"""Host synchronisations inside a train step: torch.cuda.set_sync_debug_mode("warn") around two
steps of mode F (B = 2 @ 1024x2048 to stay quick) for bf16 images and for fp32 images with fp16
compute; every warning (a blocking copy, .item(), a sync-ing op) is printed with its frame.

  python tools/sync_probe.py
"""
import os
import sys
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    from denseclip_vit_multimodal_amd.train import synth_batch, make_optimizer
    dev = torch.device("cuda", 0)
    silog = SILogLoss()
    for name, cdt, idt in [("bf16", None, torch.bfloat16), ("fp16", torch.float16, torch.float32)]:
        model = bench.make_model(dev, "F")
        if cdt is not None:
            model.backbone.compute_dtype = cdt
        model.train()
        opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
        batch = synth_batch(2, 1024, 2048, dev, 0, image_dtype=idt)
        bench.run_steps(model, opt, batch, 3, silog)  # captures, allocations, first-call setup
        torch.cuda.synchronize()
        seen = {}
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            torch.cuda.set_sync_debug_mode("warn")
            try:
                bench.run_steps(model, opt, batch, 2, silog)
            finally:
                torch.cuda.set_sync_debug_mode("default")
        torch.cuda.synchronize()
        for w in rec:
            key = (str(w.message)[:80], w.filename, w.lineno)
            seen[key] = seen.get(key, 0) + 1
        print(f"== {name}: {sum(seen.values())} synchronising calls in 2 steps", flush=True)
        for (msg, fn, ln), n in sorted(seen.items(), key=lambda kv: -kv[1]):
            print(f"  {n:3d}x {os.path.relpath(fn, ROOT)}:{ln}  {msg}")
        del model, opt, batch
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
