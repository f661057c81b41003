"""What the frozen text path (replayed on a side stream) costs a train step: mode F, B = 8 @
1024x2048 bf16, three arms in rotation on one model:
  fp32    the text encoder as built (fp32 torch modules, one HIP graph)
  bf16    the same graph captured under bf16 autocast
  const   a constant (B, 19, 512) tensor instead of the text path (measurement only)

  python tools/text_probe.py [rounds] [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    from denseclip_vit_multimodal_amd.train import synth_batch, make_optimizer
    dev = torch.device("cuda", 0)
    model = bench.make_model(dev, "F")
    model.train()
    opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
    batch = synth_batch(8, 1024, 2048, dev, 0, image_dtype=torch.bfloat16)
    silog = SILogLoss()
    cls = type(model)
    orig_fwd, orig_emb, orig_pre = cls._text_forward, cls._text_embeddings, cls._text_prelaunch

    def fwd_bf16(self, texts):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return orig_fwd(self, texts).float()

    const = {}

    def emb_const(self, B, device):
        if "t" not in const:
            const["t"] = orig_emb(self, 1, device).detach().clone()
        return const["t"].expand(B, -1, -1)

    arms = {
        "fp32": (orig_fwd, orig_emb, orig_pre),
        "bf16": (fwd_bf16, orig_emb, orig_pre),
        "const": (orig_fwd, emb_const, lambda self, device: None),
    }
    res = {k: [] for k in arms}
    for r in range(rounds):
        for name, (f, e, p) in arms.items():
            cls._text_forward, cls._text_embeddings, cls._text_prelaunch = f, e, p
            model._text_graph = None
            bench.run_steps(model, opt, batch, 3, silog)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            bench.run_steps(model, opt, batch, steps, silog)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            res[name].append(ms)
            print(f"round {r} {name:6s} {ms:8.2f} ms/step  {8e3 / ms:6.2f} img/s", flush=True)
    cls._text_forward, cls._text_embeddings, cls._text_prelaunch = orig_fwd, orig_emb, orig_pre
    for name, v in res.items():
        v = sorted(v)
        print(f"{name:6s} median {v[len(v) // 2]:8.2f} ms/step  ({', '.join(f'{x:.2f}' for x in res[name])})")
    # the text embeddings of both precisions (score map input only)
    with torch.no_grad():
        model._text_graph = None
        a = orig_emb(model, 1, dev).float()
        cls._text_forward = fwd_bf16
        model._text_graph = None
        b = orig_emb(model, 1, dev).float()
        cls._text_forward = orig_fwd
    print(f"text embeddings bf16 vs fp32: max rel {((a - b).norm() / a.norm()).item():.3e}")


if __name__ == "__main__":
    main()
