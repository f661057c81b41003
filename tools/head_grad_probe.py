"""Which input of the FCN heads' merged-tail backward (ops.MergedPointwiseFn) differs between two
fp16 runs of one seed (ViT-B/16 mode F, B = 2 @ 512x1024, exact scales, six runs of one
forward + backward): per head, hashes of dY (the head output's gradient from the fused loss
kernels), the saved input y2, dY^T X on the TN GEMM, its column sums, the torch matmul of the
merged weight gradient, and dX — and whether each product repeats bit-for-bit within a run.

  python tools/head_grad_probe.py
"""
import os, sys
sys.path.insert(0, os.getcwd())
import torch, bench
from denseclip_vit_multimodal_amd import ops, train
from denseclip_vit_multimodal_amd.train import synth_batch, make_optimizer
ops.FP16_DELAYED_SCALE = False
dev = torch.device("cuda", 0)
b1 = synth_batch(2, 512, 1024, dev, 0, image_dtype=torch.float32)
F = ops.MergedPointwiseFn
orig_f, orig_b = F.forward, F.backward
LOG = []
def fwd(ctx, y, w1, b1_, wc, bc, cdt):
    out = orig_f(ctx, y, w1, b1_, wc, bc, cdt)
    ctx.y2c = ctx.to_save[0].clone()
    ctx.tag = tuple(wc.shape)
    return out
def h(t):
    t = t.detach().float()
    return round(float(t.double().sum()), 9), round(float((t.double() * torch.arange(t.numel(), device=t.device).reshape(t.shape).double().sin()).sum()), 9)
def bwd(ctx, dout):
    y2, w1, b1_, wc, Wp = ctx.saved_tensors
    B, Cin, H, W, C1, K, Kp, in_dt, cdt = ctx.meta
    D = ops.D
    dY = D().transpose_batched(dout.contiguous(), B, K, H * W, H * W, Kp, cdt).view(B * H * W, Kp)
    G1, cs1 = ops.weight_grad(dY, y2, scale=ctx.hsb)
    G2, cs2 = ops.weight_grad(dY, y2, scale=ctx.hsb)
    W1m = w1.detach().reshape(C1, Cin).float()
    a1 = G1[:K] @ W1m.t()
    a2 = G1[:K] @ W1m.t()
    dX = ops.gemm(dY, ops.transpose2d(Wp, cdt))
    LOG.append(dict(tag=ctx.tag, G_rep=torch.equal(G1, G2), cs_rep=torch.equal(cs1, cs2), mm_rep=torch.equal(a1, a2),
                    dY=h(dY), y2=h(y2), G=h(G1), cs=h(cs1), mm=h(a1), dX=h(dX), hsb=None if ctx.hsb is None else ctx.hsb.tolist()))
    return orig_b(ctx, dout)
F.forward = staticmethod(fwd)
F.backward = staticmethod(bwd)
ref = None
for r in range(6):
    torch.manual_seed(0)
    m = bench.make_model(dev, "F").train()
    m.backbone.compute_dtype = torch.float16
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout): mod.p = 0.0
    img, seg, depth, mask = b1
    LOG.clear()
    out = m(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True)
    loss = train.loss_fn(out, seg, depth, mask)
    loss.backward()
    torch.cuda.synchronize()
    g = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    if ref is None:
        ref = g
    nd = sum(not torch.equal(g[n], ref[n]) for n in ref)
    print("run", r, "grads differing from run 0:", nd, flush=True)
    for e in LOG:
        print("    ", e, flush=True)
