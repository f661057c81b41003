"""Diagnostic: what the frozen text path (CLIPTextContextEncoder on the 19 class prompts, replayed
from a HIP graph on a side stream every step, denseclip.py _text_prelaunch) costs inside the
bench step.  Times the default bench step, then the same model with the text replay replaced by
its cached output (NOT a valid benchmark configuration: the reference recomputes the text path
every step; this only prices it), then the graph replay alone on a quiet GPU.

  python tools/text_cost.py [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    from denseclip_vit_multimodal_amd.train import synth_batch, make_optimizer
    silog = SILogLoss()
    batch = synth_batch(8, 1024, 2048, dev, 0, image_dtype=torch.bfloat16)
    model = bench.make_model(dev, "F")
    model.train()
    opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
    res = []
    for rnd in range(2):
        dt, _, _ = bench.timed(model, opt, batch, steps, 2, silog, 1)
        res.append(("default (text graph replayed every step)", dt / steps * 1e3))
        # cached text embeddings: the prelaunch does nothing and _text_embeddings returns the
        # graph's last output
        g = model._text_graph
        orig_pre, orig_emb = model._text_prelaunch, model._text_embeddings
        model._text_prelaunch = lambda device: None
        model._text_embeddings = lambda B, device: g[2].expand(B, -1, -1)
        dt2, _, _ = bench.timed(model, opt, batch, steps, 2, silog, 1)
        res.append(("text path cached (diagnostic only)", dt2 / steps * 1e3))
        model._text_prelaunch, model._text_embeddings = orig_pre, orig_emb
    torch.cuda.synchronize()
    g = model._text_graph
    for _ in range(3):
        g[1].replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        g[1].replay()
    torch.cuda.synchronize()
    res.append(("text graph replay alone", (time.perf_counter() - t0) / 20 * 1e3))
    for name, ms in res:
        print(f"{name:45s} {ms:8.2f} ms")


if __name__ == "__main__":
    main()
