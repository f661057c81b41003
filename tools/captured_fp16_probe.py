"""Where does a replayed fp16 train step (train.CapturedTrainStep) part from the eager one?

Two eager runs and one capture of the tiny context-decoder model in fp16 (fp32 images, exact
gradient scales, dropout off), the same batches; after the first replayed step the gradients of
every parameter are compared with both eager runs' gradients of that step (the eager pair gives the
run-to-run spread).  CapturedTrainStep refuses fp16 models, so the probe lifts the refusal for its
own instance.  Prints the parameters whose replay-vs-eager difference most exceeds the spread.

  python tools/captured_fp16_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from helpers import CITYSCAPES_CLASSES, TINY_CTX_CFG  # noqa: E402


def make():
    from denseclip_vit_multimodal_amd import DenseCLIP
    from denseclip_vit_multimodal_amd.train import freeze_for_mode, make_optimizer
    torch.manual_seed(0)
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **TINY_CTX_CFG).to("cuda").train()
    m.backbone.compute_dtype = torch.float16
    for mod in m.modules():
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    return m, make_optimizer(freeze_for_mode(m, "F"), capturable=True)


def main():
    from denseclip_vit_multimodal_amd import ops, train
    from denseclip_vit_multimodal_amd.train import CapturedTrainStep, synth_batch, train_step
    ops.FP16_DELAYED_SCALE = False
    dev = torch.device("cuda")
    b1 = synth_batch(2, 128, 256, dev, 0, image_dtype=torch.float32)
    b2 = synth_batch(2, 128, 256, dev, 1, image_dtype=torch.float32)
    eager = []
    for _ in range(2):
        m, o = make()
        losses = [float(train_step(m, o, b)) for b in (b1, b1, b1)]
        # step 4 (b2): its gradients, taken before the optimizer applies them
        img, seg, depth, mask = b2
        out = m(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True)
        loss = train.loss_fn(out, seg, depth, mask)
        o.zero_grad(set_to_none=True)
        loss.backward()
        torch.cuda.synchronize()
        losses.append(float(loss))
        eager.append(({n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}, losses))
    m, o = make()
    saved = train.fp16_backward
    train.fp16_backward = lambda *a, **k: False  # lift the refusal (inside __init__ only)
    try:
        cap = CapturedTrainStep(m, o, b1)
    finally:
        train.fp16_backward = saved
    # capture ran three eager warm-up steps on b1; the first replay is step 4 on b2.  The replay
    # also applies AdamW, but the gradients it produced stay in p.grad
    l4 = float(cap(b2))
    torch.cuda.synchronize()
    g = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    print("losses eager A", eager[0][1], "eager B", eager[1][1], "replay step 4", l4)
    ga, gb = eager[0][0], eager[1][0]
    print("grads", len(g), len(ga), "missing", sorted(set(ga) ^ set(g))[:5])
    rows = []
    for n in ga:
        if n not in g:
            continue
        sc = float(ga[n].abs().max()) + 1e-30
        spread = float((ga[n] - gb[n]).abs().max()) / sc
        dr = float((g[n] - ga[n]).abs().max()) / sc
        rows.append((dr / (spread + 1e-7), dr, spread, n))
    rows.sort(reverse=True)
    for r in rows[:25]:
        print(f"ratio {r[0]:10.3g}  replay-vs-eager {r[1]:.3e}  eager spread {r[2]:.3e}  {r[3]}")


if __name__ == "__main__":
    main()
