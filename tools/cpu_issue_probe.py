"""How much host time a train step needs to issue its launches (the margin the GPU-bound step
has over a slower host): mode F at B = 1 @ 1024x2048 (GPU work ~1/8 of the bench step, same
launch count), bf16 and fp16 lines; wall per step over 10 steps with one sync at the end, and
the host time spent inside the step calls.

  python tools/cpu_issue_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    from denseclip_vit_multimodal_amd.train import synth_batch, make_optimizer, train_step
    dev = torch.device("cuda", 0)
    silog = SILogLoss()
    for name, cdt, idt, B in [("bf16", None, torch.bfloat16, 1), ("fp16", torch.float16, torch.float32, 1),
                              ("bf16", None, torch.bfloat16, 8), ("fp16", torch.float16, torch.float32, 8)]:
        model = bench.make_model(dev, "F")
        if cdt is not None:
            model.backbone.compute_dtype = cdt
        model.train()
        opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
        batch = synth_batch(B, 1024, 2048, dev, 0, image_dtype=idt)
        bench.run_steps(model, opt, batch, 3, silog)
        torch.cuda.synchronize()
        host = 0.0
        t0 = time.perf_counter()
        for _ in range(10):
            h0 = time.perf_counter()
            train_step(model, opt, batch, silog)
            host += time.perf_counter() - h0
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 10 * 1e3
        print(f"{name} B={B}: wall {wall:8.2f} ms/step, host inside the step calls {host / 10 * 1e3:8.2f} ms/step",
              flush=True)
        del model, opt, batch
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
