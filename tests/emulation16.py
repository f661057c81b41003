"""16-bit emulations of the HIP ViT path for deriving gradient bounds — TEST INFRASTRUCTURE.

The fp32 oracle (oracle/denseclip_oracle.py, pinned to the reference) says what the gradients
ARE; these functions say how far ANY implementation that stores the tensors the HIP path stores
in 16 bits must land from it.  They recompute the oracle's graph in fp32 with the values rounded
at the points where the HIP kernels round them, forward and backward, so a test can hold each
HIP gradient to a multiple of the emulated error instead of a hand-picked tolerance.

Rounding points (ops.PatchEmbedFn / ops.BlockFn / ops.ReadoutFn, csrc/attention.hip):
  forward   patches and every weight (WEIGHTS copies); LN outputs xh1 / xh2; qkv; P before P.V
            (unnormalised, fp32 row sums); o; z and h = QuickGELU(z); 16-bit read-out maps
  backward  the embedding gradient (dclip_tokens_bwd's cast); the MLP branch's gradient dy (the
            cast or, with the read-out fold, dclip_layernorm_bwd_add's copy); dz (EPI_GELU_BWD
            output); dxh2 / dxh1 when LN_DY_LP (the dX GEMMs write 16 bits for the LN backward:
            bf16, or fp16 on the operand's gradient scale); the attention branch's gradient dyo (the LN backward's lp copy); dO (the
            out-projection dX GEMM output); dS and P inside the attention backward; the one-pass
            attention backward's dQ partials (one per 256 keys, DQ_KEY_BLOCK); dqkv
  fp32      residual stream, LN statistics and backward, softmax statistics, every accumulation
fp16 gradients are rounded on a per-tensor power-of-two scale (16 / max|g|, ops.grad_scale; the
attention backward's dS on its own scale, as DsScale keeps it out of the subnormals), so the
emulation models the 10-bit mantissa, not underflow the kernels avoid.

reference: segmentation/denseclip/models.py:243-294 (LN, QuickGELU, the block), 543-597 (ViT)
"""
import math

import torch
import torch.nn.functional as F

from oracle import denseclip_oracle as O


def rnd(t, dt, scaled=False):
    """t rounded to dt (returned as fp32); scaled: through a power-of-two scale to max|t| = 16."""
    if not scaled or dt != torch.float16:
        return t.to(dt).float()
    a = float(t.abs().max())
    if a == 0.0 or not math.isfinite(a):
        return t.to(dt).float()
    s = 2.0 ** math.floor(math.log2(16.0 / a))
    return (t * s).to(dt).float() / s


class Round(torch.autograd.Function):
    """16-bit storage of a value and of its gradient."""

    @staticmethod
    def forward(ctx, x, dt):
        ctx.dt = dt
        return rnd(x, dt)

    @staticmethod
    def backward(ctx, g):
        return rnd(g, ctx.dt, scaled=True), None


class RoundFwd(torch.autograd.Function):
    """16-bit value, fp32 gradient (a GEMM operand whose input gradient the kernels keep in fp32)."""

    @staticmethod
    def forward(ctx, x, dt):
        return rnd(x, dt)

    @staticmethod
    def backward(ctx, g):
        return g, None


class RoundBwd(torch.autograd.Function):
    """fp32 value, 16-bit gradient (a residual branch whose incoming gradient is cast once)."""

    @staticmethod
    def forward(ctx, x, dt):
        ctx.dt = dt
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return rnd(g, ctx.dt, scaled=True), None


# the attention backward's dQ partial granularity (keys per 16-bit partial; 0: the two-pass backward,
# whose dQ pass sums every key in fp32): the default CLS-split path since round 6 is the one-pass
# backward (DCLIP_OPT_ATTN_BWD_BLOCK 0), 256 keys per partial, for N >= 257
DQ_KEY_BLOCK = 256


class Attn16(torch.autograd.Function):
    """softmax(q k^T d^-0.5) v on (BH, N, d) fp32 tensors holding 16-bit values, with the flash
    kernels' rounding points: P (unnormalised, against the row maximum) rounded before P.V and
    normalised by its fp32 row sum; backward recomputes P from the fp32 scores, takes
    delta = rowsum(dO * O) from the stored (rounded) O, and rounds dS for dQ / dK and P for dV."""

    @staticmethod
    def forward(ctx, q, k, v, dt, o_rounded):
        s = (q @ k.transpose(1, 2)) * q.shape[-1] ** -0.5
        m = s.amax(-1, keepdim=True)
        p = torch.exp(s - m)
        l = p.sum(-1, keepdim=True)
        o = (rnd(p, dt) @ v) / l
        ctx.save_for_backward(q, k, v, m + torch.log(l), rnd(o, dt) if o_rounded else o)
        ctx.dt = dt
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, lse, o = ctx.saved_tensors
        dt = ctx.dt
        sc = q.shape[-1] ** -0.5
        p = torch.exp((q @ k.transpose(1, 2)) * sc - lse)
        dp = do @ v.transpose(1, 2)
        delta = (do * o).sum(-1, keepdim=True)
        ds = rnd(p * (dp - delta), dt, scaled=True)
        dq = (ds @ k) * sc
        n = q.shape[1]
        if DQ_KEY_BLOCK and n >= 257:
            # the one-pass backward (attention_bwd1.hip): queries 1.. sum 16-bit partials over key blocks
            # 1 + DQ_KEY_BLOCK j .. (one rounding each) plus key 0's exact term; query 0 is exact
            kb = DQ_KEY_BLOCK
            rest = ds[:, 1:, :1] @ k[:, :1] * sc
            for j0 in range(1, n, kb):
                rest = rest + rnd((ds[:, 1:, j0:j0 + kb] @ k[:, j0:j0 + kb]) * sc, dt)
            dq = torch.cat([dq[:, :1], rest], 1)
        dk = (ds.transpose(1, 2) @ q) * sc
        dv = rnd(p, dt).transpose(1, 2) @ do
        return dq, dk, dv, None, None


def block16(x, p, pre, heads, dt, ln_dy_lp):
    """ResidualAttentionBlock.forward (models.py:291-294) on x (L, B, C) with ops.BlockFn's
    rounding points."""
    L, B, C = x.shape
    d = C // heads
    r = lambda t: Round.apply(t, dt)  # noqa: E731
    rf = lambda t: RoundFwd.apply(t, dt)  # noqa: E731
    rb = lambda t: RoundBwd.apply(t, dt)  # noqa: E731
    rln = r if ln_dy_lp else rf
    h = rln(O.layer_norm(x, p[pre + "ln_1.weight"], p[pre + "ln_1.bias"]))
    qkv = r(O.linear(h, rf(p[pre + "attn.in_proj_weight"]), p[pre + "attn.in_proj_bias"]))
    q, k, v = (t.reshape(L, B * heads, d).transpose(0, 1) for t in qkv.split(C, dim=-1))
    o = Attn16.apply(q, k, v, dt, True)
    o = r(o.transpose(0, 1).reshape(L, B, C))
    x = x + rb(O.linear(o, rf(p[pre + "attn.out_proj.weight"]), p[pre + "attn.out_proj.bias"]))
    h = rln(O.layer_norm(x, p[pre + "ln_2.weight"], p[pre + "ln_2.bias"]))
    z = r(O.linear(h, rf(p[pre + "mlp.c_fc.weight"]), p[pre + "mlp.c_fc.bias"]))
    h = rf(O.quick_gelu(z))
    return x + rb(O.linear(h, rf(p[pre + "mlp.c_proj.weight"]), p[pre + "mlp.c_proj.bias"]))


def vit_forward16(img, p, dt, pre="backbone.", patch=16, heads=12, layers=12, out_indices=None, map_dt=None,
                  ln_dy_lp=None):
    """oracle.vit_forward (models.py:543-597) with the HIP path's 16-bit rounding points (module
    docstring).  map_dt: the read-out maps' dtype (None: fp32 maps, the backbone's default for fp32
    images; a 16-bit dtype: maps stored and their gradients arriving in it, DenseCLIP's HIP-neck
    path).  ln_dy_lp: the 16-bit LN-backward inputs (default: ops.LN_DY_LP for bf16, ops.LN_DY_LP_FP16
    at the fast LN widths 512 / 768 / 1024 for fp16 — on the gradient scale its GEMM operand carries)."""
    if out_indices is None:
        out_indices = [layers - 1]
    if ln_dy_lp is None:
        from denseclip_vit_multimodal_amd import ops
        if dt == torch.bfloat16:
            ln_dy_lp = ops.LN_DY_LP
        else:
            ln_dy_lp = ops.LN_DY_LP_FP16 and p[pre + "ln_pre.weight"].shape[0] in (512, 768, 1024)
    B = img.shape[0]
    rf = lambda t: RoundFwd.apply(t, dt)  # noqa: E731
    x = RoundBwd.apply(F.conv2d(rf(img), rf(p[pre + "conv1.weight"]), stride=patch), dt)
    C, H, W = x.shape[1:]
    x = x.flatten(2).transpose(1, 2)
    x = torch.cat([p[pre + "class_embedding"].expand(B, 1, -1), x], dim=1)
    x = x + O.interp_pos(p[pre + "positional_embedding"], H, W)
    x = O.layer_norm(x, p[pre + "ln_pre.weight"], p[pre + "ln_pre.bias"]).permute(1, 0, 2)
    outs = []
    for i in range(layers):
        if i > max(out_indices):
            break
        x = block16(x, p, f"{pre}transformer.resblocks.{i}.", heads, dt, ln_dy_lp)
        if i in out_indices:
            t = x.permute(1, 0, 2)
            if i == layers - 1:
                t = O.layer_norm(t, p[pre + "ln_post.weight"], p[pre + "ln_post.bias"])
            t = t[:, 1:, :].permute(0, 2, 1).reshape(B, C, H, W)
            outs.append(Round.apply(t, map_dt) if map_dt is not None else t)
    return outs


def neck_heads16(maps, p, training, dt):
    """oracle.neck / oracle.fcn_head (models.py:761-782, 13-20; FCNHead + classifier) with the HIP
    neck / heads' rounding points: 16-bit conv weights (WEIGHTS copies), conv outputs, BN + ReLU
    outputs and head logits, forward and backward; the heads' two trailing 1x1 convs as the one
    merged 16-bit weight the HIP GEMM uses (ops.MergedPointwiseFn)."""
    r = lambda t: Round.apply(t, dt)  # noqa: E731
    rw = lambda w: RoundFwd.apply(w, dt)  # noqa: E731

    def cbr(x, pre, pad):
        y = r(F.conv2d(x, rw(p[pre + "0.weight"]), padding=pad))
        return r(torch.relu(O.batch_norm(y, p, pre + "1.", training)))

    y = cbr(torch.cat([cbr(m, f"neck.process_layers.{i}.", 1) for i, m in enumerate(maps)], 1), "neck.fusion_layer.", 0)

    def head(pre):
        z = r(F.conv2d(y, rw(p[pre + "0.weight"]), padding=1))
        z = r(torch.relu(O.batch_norm(z, p, pre + "1.", training)))
        w1, wc = p[pre + "4.weight"], p[pre + "classifier.weight"]
        K, C1, Cin = wc.shape[0], w1.shape[0], w1.shape[1]
        wm = wc.reshape(K, C1) @ w1.reshape(C1, Cin)
        bm = wc.reshape(K, C1) @ p[pre + "4.bias"] + p[pre + "classifier.bias"]
        return r(F.conv2d(z, RoundFwd.apply(wm, dt).view(K, Cin, 1, 1), bm))
    return head("decode_head."), head("depth_head.")
