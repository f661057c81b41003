"""Run-to-run reproducibility of the training step.

Round 5 traced the fp16 step's run-to-run divergence (2 of 6 three-step runs, profiles/r05/r5at)
to float atomics in the fused upsample + CE / SILog gradient folds (the depth head's incoming
gradient differed in its last bits, r5ax).  ABI 7 folds every loss sum and low-res gradient in a
fixed order (csrc/headloss.hip), the small weight-gradient column sums write per-split partials
(csrc/gemm.hip colsum_kernel), and the score map's class-embedding norms are wave sums: the whole
ViT-B/16 mode-F step — backbone, HIP neck / heads, fused losses, fused AdamW — is now a fixed
computation.  Two fresh models from one seed, three steps each, must agree BIT FOR BIT in every
loss, parameter and buffer, in both 16-bit compute dtypes (fp16 with its delayed gradient
scales, as the bench runs it)."""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _run(cdt, steps=3, B=2, H=512, W=1024):
    import bench
    from denseclip_vit_multimodal_amd.train import make_optimizer, synth_batch, train_step
    torch.manual_seed(0)
    m = bench.make_model(DEV, "F").train()
    m.backbone.compute_dtype = cdt
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    assert m.fused_head_loss  # the fused resize + loss kernels are on the measured path
    opt = make_optimizer([p for p in m.parameters() if p.requires_grad])
    batch = synth_batch(B, H, W, DEV, 0, image_dtype=torch.float32 if cdt == torch.float16 else torch.bfloat16)
    losses = [train_step(m, opt, batch) for _ in range(steps)]
    torch.cuda.synchronize()
    return ([float(x) for x in losses], {n: p.detach().clone() for n, p in m.named_parameters()},
            {n: b.clone() for n, b in m.named_buffers()})


@pytest.mark.parametrize("cdt", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_three_train_steps_are_bitwise_reproducible(cdt):
    la, pa, ba = _run(cdt)
    lb, pb, bb = _run(cdt)
    assert all(x == x for x in la), la  # finite losses
    assert la == lb, (la, lb)
    diff = [n for n in pa if not torch.equal(pa[n], pb[n])]
    assert not diff, (len(diff), diff[:8])
    dbuf = [n for n in ba if not torch.equal(ba[n], bb[n])]
    assert not dbuf, dbuf[:8]


@pytest.mark.parametrize("ldt", [torch.int64, torch.uint8])
def test_fused_head_losses_are_bitwise_reproducible(ldt):
    """The fused resize + CE / SILog kernels alone, at the benchmark's head resolution (64 x 128
    low-res maps -> 1024 x 2048), ten launches each: one loss and one gradient, bit for bit."""
    from denseclip_vit_multimodal_amd import _torch_ops
    D = _torch_ops.load()
    g = torch.Generator(device="cpu").manual_seed(7)
    B, h, w, Hh, Ww = 2, 64, 128, 1024, 2048
    logits = torch.randn(B, 19, h, w, generator=g).to(DEV)
    lab = torch.randint(0, 19, (B, Hh, Ww), generator=g)
    lab[torch.rand(B, Hh, Ww, generator=g) < 0.1] = 255
    lab = lab.to(ldt).to(DEV)
    pred = (1 + 10 * torch.rand(B, 1, h, w, generator=g)).to(DEV)
    tgt = (1 + 79 * torch.rand(B, Hh, Ww, generator=g)).to(DEV)
    mask = (torch.rand(B, Hh, Ww, generator=g) >= 0.2).to(torch.uint8).to(DEV)
    ref = None
    for _ in range(10):
        s, c, gr = D.upsample_ce(logits, lab, 255)
        ss = D.upsample_silog_sums(pred, tgt, mask, 1e-6)
        gd = D.upsample_silog_grad(pred, tgt, mask, ss, 1e-6, 0.5)
        cur = (s, c, gr, ss, gd)
        if ref is None:
            ref = cur
        else:
            for a, b in zip(ref, cur):
                assert torch.equal(a, b)


def test_captured_fp16_train_step_equals_eager_exact_scales():
    """train.CapturedTrainStep with an fp16 backward (the refusal is lifted now
    that the step is reproducible): the captured step takes exact gradient scales, so it is held
    BIT FOR BIT to eager steps with ops.FP16_DELAYED_SCALE = False — ViT-B/16 mode F at 2 x 256 x
    512, fp32 images, five eager steps against three warm-up steps + two replays (the second on a
    new batch copied into the captured buffers)."""
    import bench
    from denseclip_vit_multimodal_amd import ops
    from denseclip_vit_multimodal_amd.train import CapturedTrainStep, make_optimizer, synth_batch, train_step

    def make():
        torch.manual_seed(0)
        m = bench.make_model(DEV, "F").train()
        m.backbone.compute_dtype = torch.float16
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
        return m, make_optimizer([p for p in m.parameters() if p.requires_grad], capturable=True)

    b1 = synth_batch(2, 256, 512, DEV, 0, image_dtype=torch.float32)
    b2 = synth_batch(2, 256, 512, DEV, 1, image_dtype=torch.float32)
    saved = ops.FP16_DELAYED_SCALE
    ops.FP16_DELAYED_SCALE = False
    try:
        ma, oa = make()
        la = [float(train_step(ma, oa, b)) for b in (b1, b1, b1, b2, b1)]
        mb, ob = make()
        cap = CapturedTrainStep(mb, ob, b1)  # three eager warm-up steps on b1
        lb = [float(cap(b2)), float(cap(b1))]
        torch.cuda.synchronize()
    finally:
        ops.FP16_DELAYED_SCALE = saved
    assert lb == la[3:], (lb, la)
    pa = dict(ma.named_parameters())
    diff = [n for n, p in mb.named_parameters() if not torch.equal(p, pa[n])]
    assert not diff, (len(diff), diff[:8])
