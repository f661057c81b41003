"""CPU restatement of the reference DenseCLIP ViT hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import it, and only as the checker / the timed
CPU baseline; the product package never imports it (a test enforces that).

It restates, as plain fp32 functions over a reference-named state dict, what the
reference computes (file:line in /root/reference/segmentation):

  layer_norm         denseclip/models.py:243-249   (LN in fp32, eps 1e-5, affine)
  quick_gelu         denseclip/models.py:252-254   (x * sigmoid(1.702 x))
  mha                denseclip/models.py:287-289 -> torch F.multi_head_attention_forward
                     (packed in_proj [q;k;v] with bias, scale d^-0.5, optional
                     additive mask, out_proj)
  residual_block     denseclip/models.py:291-294
  bilinear_resize    torch F.interpolate(mode='bilinear', align_corners=False) as used at
                     models.py:529-532, denseclip.py:847/899 (half-pixel source index,
                     clamped at 0, right neighbour clamped to the edge)
  interp_pos         denseclip/models.py:514-540
  vit_forward        denseclip/models.py:543-597 (patchify conv, CLS, pos, ln_pre,
                     12 blocks, per-layer NCHW read-out, ln_post only for i == L-1)
  text_context_enc   denseclip/models.py:844-864 (+ Transformer.forward applying the
                     blocks TWICE, models.py:305-307; causal mask 691-693/836-842)
  score_map          denseclip/denseclip.py:591-620, 670-675
  neck               denseclip/models.py:761-782 (ConvBNReLU 13-20)
  fcn_head           torchvision FCNHead + replaced classifier (denseclip.py:305-309,343-349)
  denseclip_forward  denseclip/denseclip.py:702-916

Parity is pinned: `tests/test_oracle_golden.py` checks this module against fixtures
produced by running the reference itself (tests/golden/gen_golden.py).
"""
import math

import torch
import torch.nn.functional as F

LN_EPS = 1e-5

# When True, the unmasked attention core uses torch's scaled_dot_product_attention — the
# very op the reference reaches through nn.MultiheadAttention (CPU flash kernel, no N x N
# buffer).  bench.py's cpu_baseline sets it so fwd+bwd at N = 8193 fits in host memory;
# the parity tests keep the explicit softmax restatement (False).
USE_SDPA = False


# ----------------------------------------------------------------------------- primitives
def layer_norm(x, w, b, eps=LN_EPS):
    """models.py:243-249 — statistics and affine in fp32, biased variance."""
    xf = x.float()
    mu = xf.mean(-1, keepdim=True)
    var = ((xf - mu) ** 2).mean(-1, keepdim=True)
    y = (xf - mu) / torch.sqrt(var + eps) * w.float() + b.float()
    return y.to(x.dtype)


def quick_gelu(x):
    """models.py:252-254."""
    return x * torch.sigmoid(1.702 * x)


def linear(x, w, b=None):
    y = x @ w.t()
    return y + b if b is not None else y


def mha(x, in_w, in_b, out_w, out_b, heads, attn_mask=None, q_chunk=1024):
    """nn.MultiheadAttention(x, x, x, need_weights=False) on x (L, B, C) (models.py:287-289).

    Softmax is evaluated in query chunks so that L = 8193 fits in memory; the math is
    the plain softmax(q k^T * d^-0.5 + mask) v.
    """
    L, B, C = x.shape
    d = C // heads
    qkv = linear(x, in_w, in_b)                                   # (L, B, 3C)
    q, k, v = qkv.split(C, dim=-1)
    q = q.reshape(L, B * heads, d).transpose(0, 1)                # (BH, L, d)
    k = k.reshape(L, B * heads, d).transpose(0, 1)
    v = v.reshape(L, B * heads, d).transpose(0, 1)
    scale = d ** -0.5
    if USE_SDPA and attn_mask is None:
        out = F.scaled_dot_product_attention(q, k, v)
        return linear(out.transpose(0, 1).reshape(L, B, C), out_w, out_b)
    out = torch.empty_like(q)
    for s in range(0, L, q_chunk):
        e = min(L, s + q_chunk)
        sc = (q[:, s:e] * scale) @ k.transpose(1, 2)
        if attn_mask is not None:
            sc = sc + attn_mask[s:e]
        out[:, s:e] = torch.softmax(sc, dim=-1) @ v
    out = out.transpose(0, 1).reshape(L, B, C)
    return linear(out, out_w, out_b)


def residual_block(x, p, pre, heads, attn_mask=None):
    """ResidualAttentionBlock.forward (models.py:291-294), x in LND."""
    h = layer_norm(x, p[pre + "ln_1.weight"], p[pre + "ln_1.bias"])
    x = x + mha(h, p[pre + "attn.in_proj_weight"], p[pre + "attn.in_proj_bias"],
                p[pre + "attn.out_proj.weight"], p[pre + "attn.out_proj.bias"], heads, attn_mask)
    h = layer_norm(x, p[pre + "ln_2.weight"], p[pre + "ln_2.bias"])
    h = quick_gelu(linear(h, p[pre + "mlp.c_fc.weight"], p[pre + "mlp.c_fc.bias"]))
    return x + linear(h, p[pre + "mlp.c_proj.weight"], p[pre + "mlp.c_proj.bias"])


def _src_index(out_size, in_size):
    """PyTorch's align_corners=False source coordinate: (dst+0.5)*in/out-0.5, clamp>=0."""
    scale = in_size / out_size
    dst = torch.arange(out_size, dtype=torch.float64)
    src = ((dst + 0.5) * scale - 0.5).clamp(min=0.0)
    i0 = src.floor().long().clamp(max=in_size - 1)
    i1 = torch.where(i0 < in_size - 1, i0 + 1, i0)
    l1 = (src - i0.double()).float()
    return i0, i1, 1.0 - l1, l1


def bilinear_resize(x, out_h, out_w):
    """Bilinear, align_corners=False, x (N, C, H, W) -> (N, C, out_h, out_w).

    Note: PyTorch computes the coordinates in float32 (area_pixel_compute_source_index
    with an fp32 scale); the fp64 coordinates here agree with it to the last ulp for the
    power-of-two scales on this path and within 1e-6 otherwise.
    """
    N, C, H, W = x.shape
    y0, y1, wy0, wy1 = _src_index(out_h, H)
    x0, x1, wx0, wx1 = _src_index(out_w, W)
    top = x[:, :, y0, :] * wy0.view(1, 1, -1, 1) + x[:, :, y1, :] * wy1.view(1, 1, -1, 1)
    return top[:, :, :, x0] * wx0.view(1, 1, 1, -1) + top[:, :, :, x1] * wx1.view(1, 1, 1, -1)


def interp_pos(pos, H, W):
    """interpolate_pos_encoding (models.py:514-540): (g*g+1, C) -> (H*W+1, C)."""
    n_loaded = pos.shape[0] - 1
    if H * W == n_loaded:
        return pos
    g = int(math.isqrt(n_loaded))
    C = pos.shape[1]
    grid = pos[1:].reshape(1, g, g, C).permute(0, 3, 1, 2)
    grid = bilinear_resize(grid, H, W)
    return torch.cat([pos[:1], grid.permute(0, 2, 3, 1).reshape(H * W, C)], dim=0)


# ----------------------------------------------------------------------------- ViT
def vit_forward(img, p, pre="backbone.", patch=16, heads=12, layers=12, out_indices=None):
    """CLIPVisionTransformer.forward (models.py:543-597).  Returns the list of maps."""
    if out_indices is None:
        out_indices = [layers - 1]
    B = img.shape[0]
    x = F.conv2d(img, p[pre + "conv1.weight"], stride=patch)       # (B, C, H, W)
    C, H, W = x.shape[1:]
    x = x.flatten(2).transpose(1, 2)                                # NLC
    cls = p[pre + "class_embedding"].to(x.dtype).expand(B, 1, -1)
    x = torch.cat([cls, x], dim=1)
    x = x + interp_pos(p[pre + "positional_embedding"], H, W).to(x.dtype)
    x = layer_norm(x, p[pre + "ln_pre.weight"], p[pre + "ln_pre.bias"])
    x = x.permute(1, 0, 2)                                          # LND
    outs = []
    for i in range(layers):
        x = residual_block(x, p, f"{pre}transformer.resblocks.{i}.", heads)
        if i in out_indices:
            t = x.permute(1, 0, 2)
            if i == layers - 1:
                t = layer_norm(t, p[pre + "ln_post.weight"], p[pre + "ln_post.bias"])
            outs.append(t[:, 1:, :].permute(0, 2, 1).reshape(B, C, H, W))
    return outs


# ----------------------------------------------------------------------------- text path
def causal_mask(n):
    m = torch.full((n, n), float("-inf"))
    return m.triu_(1)


def text_context_encoder(tokens, contexts, p, pre="text_encoder.", heads=8, layers=12):
    """CLIPTextContextEncoder.forward (models.py:844-864)."""
    tok_emb = p[pre + "token_embedding.weight"][tokens]            # (K, N1, C)
    K, N1, C = tok_emb.shape
    B, N2, _ = contexts.shape
    eos = tokens.argmax(dim=-1) + N2
    eos = eos.reshape(1, K).expand(B, K).reshape(-1)
    xt = tok_emb.reshape(1, K, N1, C).expand(B, K, N1, C)
    ctx = contexts.reshape(B, 1, N2, C).expand(B, K, N2, C)
    x = torch.cat([xt[:, :, 0:1], ctx, xt[:, :, 1:]], dim=2).reshape(B * K, N1 + N2, C)
    x = x + p[pre + "positional_embedding"]
    x = x.permute(1, 0, 2)
    mask = causal_mask(x.shape[0])
    # Transformer.forward runs every block, then the whole Sequential again (305-307)
    for _ in range(2):
        for i in range(layers):
            x = residual_block(x, p, f"{pre}transformer.resblocks.{i}.", heads, mask)
    x = x.permute(1, 0, 2)
    x = layer_norm(x, p[pre + "ln_final.weight"], p[pre + "ln_final.bias"])
    x = x[torch.arange(x.shape[0]), eos] @ p[pre + "text_projection"]
    return x.reshape(B, K, -1)


def _ln(x, p, pre, eps=LN_EPS):
    return layer_norm(x, p[pre + "weight"], p[pre + "bias"], eps)


def _decoder_attention(q, kv, p, pre, heads):
    """Attention.forward (models.py:328-344): bias-free q/k/v projections, per-head softmax of
    q.k * d^-0.5 over the memory, output projection (dropout = identity)."""
    B, N, C = q.shape
    M = kv.shape[1]
    qh = linear(q, p[pre + "q_proj.weight"]).reshape(B, N, heads, C // heads)
    kh = linear(kv, p[pre + "k_proj.weight"]).reshape(B, M, heads, C // heads)
    vh = linear(kv, p[pre + "v_proj.weight"]).reshape(B, M, heads, C // heads)
    a = (torch.einsum("bnkc,bmkc->bknm", qh, kh) * (C // heads) ** -0.5).softmax(dim=-1)
    x = torch.einsum("bknm,bmkc->bnkc", a, vh).reshape(B, N, C)
    return linear(x, p[pre + "proj.weight"], p[pre + "proj.bias"])


def context_decoder(text, visual, p, pre="context_decoder.", heads=4, layers=6):
    """ContextDecoder.forward (models.py:910-917) over TransformerDecoderLayer (models.py:369-375):
    memory = LN(Linear(LN(visual))), x = Linear(LN(text)); per layer x += SelfAttn(LN1 x),
    x += CrossAttn(LN2 x, memory), x += MLP(LN3 x) (exact GELU); out = Linear(LN(x))."""
    mem = _ln(linear(_ln(visual, p, pre + "memory_proj.0."), p[pre + "memory_proj.1.weight"],
                     p[pre + "memory_proj.1.bias"]), p, pre + "memory_proj.2.")
    x = linear(_ln(text, p, pre + "text_proj.0."), p[pre + "text_proj.1.weight"], p[pre + "text_proj.1.bias"])
    for i in range(layers):
        L = f"{pre}decoder.{i}."
        y = _ln(x, p, L + "norm1.")
        x = x + _decoder_attention(y, y, p, L + "self_attn.", heads)
        x = x + _decoder_attention(_ln(x, p, L + "norm2."), mem, p, L + "cross_attn.", heads)
        h = F.gelu(linear(_ln(x, p, L + "norm3."), p[L + "mlp.0.weight"], p[L + "mlp.0.bias"]))
        x = x + linear(h, p[L + "mlp.3.weight"], p[L + "mlp.3.bias"])
    return linear(_ln(x, p, pre + "out_proj.0."), p[pre + "out_proj.1.weight"], p[pre + "out_proj.1.bias"])


def l2_normalize(x, dim, eps=1e-12):
    """F.normalize(p=2): x / max(||x||, eps)."""
    n = x.norm(p=2, dim=dim, keepdim=True).clamp(min=eps)
    return x / n


def score_map(visual, text, p):
    """_process_features score map (denseclip.py:591-620, 670-675).

    visual: last backbone map (B, Cv, h, w); text: (B, K, Ct).  Returns (score, global).
    """
    g = visual.mean(dim=(2, 3))
    if "global_proj.weight" in p:
        g = linear(g, p["global_proj.weight"], p["global_proj.bias"])
    if "vis_proj.weight" in p:
        visual = F.conv2d(visual, p["vis_proj.weight"], p["vis_proj.bias"])
    vn = l2_normalize(visual, 1)
    tn = l2_normalize(text, 2)
    return torch.einsum("bchw,bkc->bkhw", vn, tn), g


# ----------------------------------------------------------------------------- neck / heads
def batch_norm(x, p, pre, training):
    w, b = p[pre + "weight"], p[pre + "bias"]
    if training:
        mu = x.mean(dim=(0, 2, 3), keepdim=True)
        var = ((x - mu) ** 2).mean(dim=(0, 2, 3), keepdim=True)
    else:
        mu = p[pre + "running_mean"].view(1, -1, 1, 1)
        var = p[pre + "running_var"].view(1, -1, 1, 1)
    return (x - mu) / torch.sqrt(var + 1e-5) * w.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


def conv_bn_relu(x, p, pre, pad, training):
    """ConvBNReLU (models.py:13-20)."""
    x = F.conv2d(x, p[pre + "0.weight"], padding=pad)
    return torch.relu(batch_norm(x, p, pre + "1.", training))


def neck(maps, p, pre="neck.", training=False):
    """ViTFeatureFusionNeck.forward (models.py:761-782)."""
    feats = [conv_bn_relu(m, p, f"{pre}process_layers.{i}.", 1, training) for i, m in enumerate(maps)]
    return conv_bn_relu(torch.cat(feats, 1), p, pre + "fusion_layer.", 0, training)


def fcn_head(x, p, pre, training=False):
    """torchvision FCNHead (conv3x3-BN-ReLU-Dropout-conv1x1) + `.classifier` conv1x1.

    The reference assigns `.classifier` onto the nn.Sequential, which appends it to the
    module sequence, so it runs after the FCNHead's own last conv (denseclip.py:307-308).
    Dropout is the identity here (eval, or train with dropout disabled).
    """
    x = F.conv2d(x, p[pre + "0.weight"], padding=1)
    x = torch.relu(batch_norm(x, p, pre + "1.", training))
    x = F.conv2d(x, p[pre + "4.weight"], p[pre + "4.bias"])
    return F.conv2d(x, p[pre + "classifier.weight"], p[pre + "classifier.bias"])


# ----------------------------------------------------------------------------- full model
def denseclip_forward(img, p, tokens, cfg, gt_hw=None, training=False):
    """DenseCLIP.forward (denseclip.py:702-916) for the ViT + context-encoder config.

    Returns a dict with the intermediates the tests compare:
      maps, text, score, seg_low, depth_low, seg, depth.
    """
    bb = cfg["backbone"]
    te = cfg["text_encoder"]
    layers = bb.get("layers", 12)
    outs = sorted(set(bb.get("out_indices") or [layers - 1]))
    maps = vit_forward(img, p, patch=bb.get("patch_size", 16), heads=bb.get("heads", 12),
                       layers=layers, out_indices=outs)
    B = img.shape[0]
    contexts = p["contexts"]
    text = text_context_encoder(tokens, contexts, p, heads=te.get("transformer_heads", 8),
                                layers=te.get("transformer_layers", 12)).expand(B, -1, -1)
    cd = cfg.get("context_decoder")
    if cd:
        # 'attention' context (denseclip.py:627-633): [projected global; projected pixels],
        # fused as text + gamma * ContextDecoder(text, context) (denseclip.py:661-665)
        vis = maps[-1]
        g = vis.mean(dim=(2, 3))
        if "global_proj.weight" in p:
            g = linear(g, p["global_proj.weight"], p["global_proj.bias"])
        if "vis_proj.weight" in p:
            vis = F.conv2d(vis, p["vis_proj.weight"], p["vis_proj.bias"])
        ctx = torch.cat([g.unsqueeze(1), vis.flatten(2).permute(0, 2, 1)], dim=1)
        text = text + p["gamma"] * context_decoder(text, ctx, p, heads=cd.get("transformer_heads", 4),
                                                   layers=cd.get("transformer_layers", 6))
    score, _ = score_map(maps[-1], text, p)
    fused = neck(maps, p, training=training)
    seg_low = fcn_head(fused, p, "decode_head.", training)
    depth_low = fcn_head(fused, p, "depth_head.", training)
    H, W = gt_hw if gt_hw is not None else img.shape[2:]
    seg = bilinear_resize(seg_low, H, W) if seg_low.shape[-2:] != (H, W) else seg_low
    depth = bilinear_resize(depth_low, H, W) if depth_low.shape[-2:] != (H, W) else depth_low
    return dict(maps=maps, text=text, score=score, seg_low=seg_low, depth_low=depth_low,
                seg=seg, depth=depth)


def silog_loss(pred, target, mask, lambd=0.5, eps=1e-6):
    """SILogLoss.forward (denseclip/losses.py:21-78)."""
    d = torch.log(pred.clamp(min=eps)) - torch.log(target.clamp(min=eps))
    d = torch.where(mask, d, torch.zeros_like(d))
    T = int(mask.sum())
    if T == 0:
        return d.sum() * 0
    return (d ** 2).sum() / T - lambd * d.sum() ** 2 / T ** 2
