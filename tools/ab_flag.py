"""A/B a module-level switch of the package on the whole train step (mode F, B = 8 @ 1024x2048,
bf16 images unless --fp16) in ONE process: the arms alternate over rounds on the same model.

  python tools/ab_flag.py ops.EAGER_WEIGHT_REFRESH True False [--rounds 3] [--steps 10] [--fp16]
  python tools/ab_flag.py opt:6 0 3      (a libdclip kernel-variant option, dclip_set_option)
"""
import argparse
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("flag")
    ap.add_argument("values", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--fp16", action="store_true")
    ap.add_argument("--fp8", action="store_true", help="the fp8 attention forward (BASELINE configs[4])")
    a = ap.parse_args()
    vals = [eval(v) for v in a.values]  # noqa: S307 (literals from the command line)
    if a.flag.startswith("opt:"):
        from denseclip_vit_multimodal_amd import _native
        oid = int(a.flag[4:])

        def setv(v):
            _native.call("dclip_set_option", oid, int(v))
    else:
        modname, attr = a.flag.rsplit(".", 1)
        mod = importlib.import_module("denseclip_vit_multimodal_amd." + modname)

        def setv(v):
            setattr(mod, attr, v)
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    from denseclip_vit_multimodal_amd.train import synth_batch, make_optimizer
    dev = torch.device("cuda", 0)
    model = bench.make_model(dev, "F")
    if a.fp16:
        model.backbone.compute_dtype = torch.float16
    if a.fp8:
        model.backbone.attn_fp8 = True
    model.train()
    opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
    batch = synth_batch(8, 1024, 2048, dev, 0, image_dtype=torch.float32 if a.fp16 else torch.bfloat16)
    silog = SILogLoss()
    res = {repr(v): [] for v in vals}
    for r in range(a.rounds):
        # the arms' order reversed every other round (ABBA): a drift of the box within a round
        # (clock, temperature) would otherwise favour the arm that always runs first
        for v in (vals if r % 2 == 0 else vals[::-1]):
            setv(v)
            bench.run_steps(model, opt, batch, 3, silog)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            bench.run_steps(model, opt, batch, a.steps, silog)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            res[repr(v)].append(ms)
            print(f"round {r} {a.flag}={v!r:8}  {ms:8.2f} ms/step  {8e3 / ms:6.2f} img/s", flush=True)
    from denseclip_vit_multimodal_amd import ops
    print("path counters:", {k: v for k, v in ops.STATS.items() if "fold" in k or "readout" in k})
    for k, v in res.items():
        s = sorted(v)
        print(f"{a.flag}={k:8} median {s[len(s) // 2]:8.2f} ms/step  ({', '.join(f'{x:.2f}' for x in v)})")


if __name__ == "__main__":
    main()
