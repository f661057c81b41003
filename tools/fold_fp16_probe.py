"""The fp16 read-out fold test's arms in one process: fold off, off again, off with the output
gradient scaled by (1 + 2^-20) (the noise floor: an fp32-ulp-sized perturbation re-rounded through
every 16-bit cast of the backward), and on — the five worst parameters' relative gradient
differences against the first run.

  python tools/fold_fp16_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from helpers import CITYSCAPES_CFG, CITYSCAPES_CLASSES, images, rel_err, spec_state_dict  # noqa: E402
from denseclip_vit_multimodal_amd import DenseCLIP, ops as O  # noqa: E402

DEV = "cuda"
m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **CITYSCAPES_CFG)
m.load_state_dict(spec_state_dict("cityscapes"))
bb, neck = m.backbone.to(DEV).train(), m.neck.to(DEV).train()
x = images(2, 128, 256).to(DEV).half()
gen = torch.Generator(device=DEV).manual_seed(4)
gout = torch.randn(2, 256, 8, 16, device=DEV, generator=gen) * 1e-4
named = [(n, p) for n, p in list(bb.named_parameters()) + [("neck." + n, p) for n, p in neck.named_parameters()]
         if p.requires_grad]
runs = []
for fold, eps in ((False, 0.0), (False, 0.0), (False, 2.0 ** -20), (True, 0.0)):
    O.FOLD_READOUT_GRAD = fold
    for blk in bb.transformer.resblocks:
        blk.__dict__.pop("_dclip_dscale", None)
    for _ in range(2):
        for _, p in named:
            p.grad = None
        out = neck(bb(x))[0]
        (out.float() * (gout * (1.0 + eps))).sum().backward()
    runs.append({n: p.grad.clone() for n, p in named if p.grad is not None})
for j, label in ((1, "off vs off"), (2, "off vs off, output gradient x (1 + 2^-20)"), (3, "off vs on")):
    errs = sorted(((rel_err(runs[j][n].float(), runs[0][n].float()), n) for n in runs[0]), reverse=True)
    print(label + ": " + ", ".join(f"{n} {e:.2e}" for e, n in errs[:5]), flush=True)
