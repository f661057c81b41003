"""DenseCLIP modules with the reference's class names, constructor kwargs and state-dict keys
(reference seg/denseclip/models.py).  The CLIPVisionTransformer forward — the hot path —
runs entirely on the HIP kernels of libdclip.so (see ops.py).  ViTFeatureFusionNeck keeps the
reference's torch module structure (its state-dict keys), but on 16-bit GPU maps its levels,
BatchNorms and fusion conv run on the HIP implicit-GEMM conv / BN kernels (ops.NeckLevelsFn,
ops.bn_train, ops.Conv1x1Fn); the text encoder and the ContextDecoder stay plain torch modules
(batch-independent; SURVEY §2 row 4-5, out of kernel scope).
"""
import logging
import math
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops

logger = logging.getLogger(__name__)


class BatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d (same parameters, buffers and state-dict keys).  16-bit channels-last maps
    run the HIP batch-norm kernels: train mode through ops.BatchNormFn, eval mode (no gradient)
    through dclip_bn_eval; everything else runs torch's native kernels instead of MIOpen: MIOpen's batch-norm segfaults on the host for a
    bf16 channels-last (1, 128, 73, 146) map in train mode — the ViT-L/14 neck at 1024x2048 —
    while fp32, NCHW, other sizes and the native kernels are fine (tools/bn_probe.py,
    gpurun_out/bn_probe.log)."""

    def forward(self, x):
        if ops.bn_hip_ok(self, x):
            # batch statistics on the HIP kernels (torch's native channels-last kernels run at
            # ~0.12 TB/s on the neck maps): dclip_bn_fwd / dclip_bn_bwd
            return ops.bn_train(self, x)
        if ops.bn_eval_ok(self, x):  # running statistics, no gradient: dclip_bn_eval
            return ops.bn_eval(self, x)
        ops.note_torch_fallback()
        if x.is_cuda:
            with torch.backends.cudnn.flags(enabled=False):
                return super().forward(x)
        return super().forward(x)


class ConvBNReLU(nn.Sequential):
    """Conv-BN-ReLU (reference models.py:13-20)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, padding=1, stride=1):
        super().__init__(
            nn.Conv2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding, bias=False),
            BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
        )


class Registry:
    """Name registry (reference models.py:48-67 / heads.py:64-79)."""

    def __init__(self):
        self._registry = {}

    def register_module(self, name=None):
        def deco(cls):
            self._registry[name or cls.__name__] = cls
            return cls
        return deco

    def get(self, name):
        return self._registry.get(name)

    def build(self, cfg, **kwargs):
        if isinstance(cfg, dict):
            cfg = dict(cfg)
            return self._registry[cfg.pop("type")](**cfg, **kwargs)
        return self._registry[cfg](**kwargs)


BACKBONES = Registry()


class LayerNorm(nn.LayerNorm):
    """LayerNorm computed in fp32 and cast back (reference models.py:243-249)."""

    def forward(self, x):
        orig = x.dtype
        return super().forward(x.type(torch.float32)).type(orig)


class QuickGELU(nn.Module):
    """x * sigmoid(1.702 x) (reference models.py:252-254)."""

    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


def drop_path(x, drop_prob=0.0, training=False, scale_by_keep=True):
    """Stochastic depth as timm.layers.drop_path (the reference's import, models.py:9): one keep
    value per index of dim 0, Bernoulli(1 - p), divided by 1 - p."""
    if drop_prob == 0.0 or not training:
        return x
    keep = 1 - drop_prob
    shape = (x.shape[0],) + (1,) * (x.ndim - 1)
    m = x.new_empty(shape).bernoulli_(keep)
    if keep > 0.0 and scale_by_keep:
        m.div_(keep)
    return x * m


class DropPath(nn.Module):
    def __init__(self, drop_prob=None):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        return drop_path(x, self.drop_prob, self.training)

    def extra_repr(self):
        return f"p={self.drop_prob}"


class ResidualAttentionBlock(nn.Module):
    """Pre-LN block (reference models.py:271-294).  `forward` is the plain-torch path used by
    the text encoder (masked, LND); the ViT drives the same parameters through the fused
    HIP block (ops.BlockFn)."""

    def __init__(self, d_model, n_head, attn_mask=None, drop_path=0.0):
        super().__init__()
        self.attn = nn.MultiheadAttention(d_model, n_head)
        self.ln_1 = LayerNorm(d_model)
        self.mlp = nn.Sequential(OrderedDict([
            ("c_fc", nn.Linear(d_model, d_model * 4)),
            ("gelu", QuickGELU()),
            ("c_proj", nn.Linear(d_model * 4, d_model)),
        ]))
        self.ln_2 = LayerNorm(d_model)
        self.attn_mask = attn_mask
        self.n_head = n_head
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()

    def attention(self, x):
        m = None
        if self.attn_mask is not None:
            # the mask is not a buffer (state-dict keys as in the reference): keep a device copy
            # instead of a host->device copy (and host sync) per call
            key = (x.device, x.dtype)
            if getattr(self, "_mask_key", None) != key:
                self._mask_dev = self.attn_mask.to(dtype=x.dtype, device=x.device)
                self._mask_key = key
            m = self._mask_dev
        return self.attn(x, x, x, need_weights=False, attn_mask=m)[0]

    def forward(self, x):
        x = x + self.drop_path(self.attention(self.ln_1(x)))
        return x + self.drop_path(self.mlp(self.ln_2(x)))

    def hip_params(self):
        return (self.ln_1.weight, self.ln_1.bias, self.attn.in_proj_weight, self.attn.in_proj_bias,
                self.attn.out_proj.weight, self.attn.out_proj.bias, self.ln_2.weight, self.ln_2.bias,
                self.mlp.c_fc.weight, self.mlp.c_fc.bias, self.mlp.c_proj.weight, self.mlp.c_proj.bias)


class Transformer(nn.Module):
    """Reference models.py:297-307.  NOTE: `forward` applies every block and then the whole
    Sequential again — the reference's behaviour, reproduced for parity (text encoder)."""

    def __init__(self, width, layers, heads, attn_mask=None, drop_path_rate=0.0):
        super().__init__()
        self.width = width
        self.layers = layers
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, layers)]
        self.resblocks = nn.Sequential(*[ResidualAttentionBlock(width, heads, attn_mask, dpr[i])
                                         for i in range(layers)])

    def forward(self, x):
        for blk in self.resblocks:
            x = blk(x)
        return self.resblocks(x)


# ============================================================================ ViT backbone
@BACKBONES.register_module()
class CLIPVisionTransformer(nn.Module):
    """CLIP ViT image encoder with per-layer dense read-out (reference models.py:378-597).

    forward(x: (B, 3, H, W)) -> list of (B, width, H // p, W // p) maps, one per
    out_index in ascending order, in x.dtype.  Runs on the HIP kernels only (x must be a
    GPU tensor).  The compute dtype of the GEMM/attention operands is bf16 for bf16 input,
    fp16 for fp16 input and `compute_dtype` for fp32 input — default fp16, the dtype that
    meets the reference within the north-star 1e-3 (fp32 images are what the reference
    trainer feeds; bf16 holds 1e-2 and is the throughput setting: feed bf16 images or set
    compute_dtype=torch.bfloat16); the residual stream and LayerNorms are fp32 throughout.  `attn_fp8=True` (BASELINE config 5) runs the
    attention forward on the e4m3 MFMA kernel (dclip_attn_fwd_fp8); its backward is the 16-bit
    flash backward recomputing P against the fp8 forward's lse.
    """

    def __init__(self, input_resolution=224, patch_size=16, width=768, layers=12, heads=12, output_dim=768,
                 drop_path_rate=0.0, out_indices=None, pretrained=None, compute_dtype=torch.float16,
                 attn_fp8=False, **kwargs):
        super().__init__()
        self.pretrained = pretrained
        self.input_resolution = input_resolution
        self.output_dim = width
        self.layers = layers
        self.width = width
        self.heads = heads
        self.patch_size = patch_size
        self.compute_dtype = compute_dtype
        self.attn_fp8 = bool(attn_fp8)
        self.drop_path_rate = drop_path_rate
        self.conv1 = nn.Conv2d(3, width, kernel_size=patch_size, stride=patch_size, bias=False)
        scale = width ** -0.5
        self.class_embedding = nn.Parameter(scale * torch.randn(width))
        self.grid_size = input_resolution // patch_size
        self.positional_embedding = nn.Parameter(scale * torch.randn(self.grid_size ** 2 + 1, width))
        self.ln_pre = LayerNorm(width)
        self.transformer = Transformer(width, layers, heads, drop_path_rate=drop_path_rate)
        self.ln_post = LayerNorm(width)
        self._clip_proj_dim = 512
        self.proj = nn.Parameter(scale * torch.randn(width, self._clip_proj_dim))
        if out_indices is None:
            self.out_indices = [layers - 1]
        else:
            if not isinstance(out_indices, (list, tuple)):
                raise TypeError("out_indices must be list or tuple")
            for i in out_indices:
                if not 0 <= i < layers:
                    raise ValueError(f"Index {i} in out_indices is out of range for {layers} layers.")
            self.out_indices = sorted(set(out_indices))
        self.init_weights()

    def _init_weights_default(self, m):
        if isinstance(m, nn.Linear):
            nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)
        elif isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)

    def init_weights(self, pretrained=None):
        """OpenAI CLIP TorchScript weights (visual.* keys), pos-embed resized bilinearly to
        this grid (reference models.py:459-512); default init otherwise."""
        pretrained = pretrained or self.pretrained
        if not isinstance(pretrained, str):
            logger.warning("No pretrained weights specified for ViT. Applying default initialization.")
            self.apply(self._init_weights_default)
            return
        try:
            ckpt = torch.jit.load(pretrained, map_location="cpu").float().state_dict()
        except FileNotFoundError:
            logger.error(f"Pretrained ViT file not found: {pretrained}")
            return
        sd = OrderedDict((k[len("visual."):], v) for k, v in ckpt.items() if k.startswith("visual."))
        if "positional_embedding" in sd and sd["positional_embedding"].shape != self.positional_embedding.shape:
            pe = sd["positional_embedding"]
            g0 = int(np.sqrt(pe.shape[0] - 1))
            if g0 * g0 != pe.shape[0] - 1:
                sd.pop("positional_embedding")
            else:
                grid = pe[1:].reshape(1, g0, g0, -1).permute(0, 3, 1, 2)
                grid = F.interpolate(grid, size=(self.grid_size, self.grid_size), mode="bilinear",
                                     align_corners=False)
                sd["positional_embedding"] = torch.cat([pe[:1], grid.permute(0, 2, 3, 1).reshape(-1, pe.shape[1])])
        if "proj" in sd and sd["proj"].shape != self.proj.shape:
            sd.pop("proj")
        msg = self.load_state_dict(sd, strict=False)
        logger.info(f"ViT weights loaded: {msg}")

    def _cdt(self, x):
        if x.dtype in (torch.bfloat16, torch.float16):
            return x.dtype
        return self.compute_dtype

    def forward(self, x, map_dtype=None):
        """map_dtype (extension; default x.dtype, the reference contract): dtype of the returned
        maps.  DenseCLIP passes the compute dtype for fp32 images so the HIP neck and heads read
        the read-out token buffers in place (their outputs are returned in fp32)."""
        if not x.is_cuda:
            raise RuntimeError("CLIPVisionTransformer runs on the MI355X HIP kernels only (got a CPU tensor)")
        if self.width != self.heads * 64:
            raise NotImplementedError(f"the fused attention kernel needs head_dim 64 (width {self.width}, "
                                      f"heads {self.heads})")
        B, _, Hin, Win = x.shape
        p = self.patch_size
        gh, gw = Hin // p, Win // p
        Ntok = gh * gw + 1
        cdt = self._cdt(x)
        tok = ops.PatchEmbedFn.apply(x, self.conv1.weight, self.class_embedding, self.positional_embedding,
                                     self.ln_pre.weight, self.ln_pre.bias, p, cdt)
        outs = []
        meta = (B, Ntok, self.heads, cdt, self.attn_fp8)
        mdt = map_dtype or x.dtype
        hsb = ops._head_scale_buf()  # the 16-bit heads' gradient scale (DenseCLIP, fp16, fp32 images)
        rmeta = (B, Ntok, gh, gw, mdt, hsb)
        last = max(self.out_indices) if self.out_indices else -1
        fp16_bwd = cdt == torch.float16 and torch.is_grad_enabled()
        link_in = None  # the previous block's ops.ReadoutLink (meta[8]): folded into this block's ln_1 backward
        for i, blk in enumerate(self.transformer.resblocks):
            if i > last:
                break  # later blocks feed nothing the reference returns
            dp = _drop_path_masks(blk, Ntok, x.device) if self.training else None
            # the fp16 backward's delayed gradient scales live on the block across steps (meta[7])
            ds = _delayed_scale(blk) if fp16_bwd else None
            if i in self.out_indices and i != self.layers - 1:
                # read-out without ln_post: produced by the block itself, so its gradient is
                # folded into the block's backward (ops.BlockFn, meta[5]) — or, bf16, into the next
                # block's ln_1 backward (meta[9], ops.ReadoutLink)
                link = None
                if ops.FOLD_READOUT_GRAD and torch.is_grad_enabled() and i < last and dp is None \
                        and self.width in (512, 768, 1024):
                    if cdt == torch.bfloat16 and mdt == torch.bfloat16 and hsb is None:
                        link = ops.ReadoutLink(gh, gw)
                    elif cdt == torch.float16 and ds is not None and ops.FP16_DELAYED_SCALE and \
                            mdt in (torch.float16, torch.bfloat16):
                        link = ops.ReadoutLink(gh, gw, ds, hsb)
                bmeta = meta + ((gh, gw, mdt, hsb), dp, ds, link_in, link)
                tok, fmap = ops.BlockFn.apply(tok, bmeta, *blk.hip_params())
                if link is not None:
                    fmap._dclip_link = link  # read by the map gradient's producer (ops.NeckLevelsFn)
                link_in = link
                outs.append(fmap)
                continue
            tok = ops.BlockFn.apply(tok, meta + (None, dp, ds, link_in, None), *blk.hip_params())
            link_in = None
            if i in self.out_indices:  # the last layer: ln_post (models.py:576)
                outs.append(ops.ReadoutFn.apply(tok, self.ln_post.weight, self.ln_post.bias, rmeta))
        return outs


def _delayed_scale(blk):
    """The block's ops.DelayedScale (created on first use; not a parameter or buffer: it is no part
    of the state dict)."""
    ds = blk.__dict__.get("_dclip_dscale")
    if ds is None:
        ds = blk.__dict__["_dclip_dscale"] = ops.DelayedScale()
    return ds


def _drop_path_masks(blk, ntok, device):
    """The two stochastic-depth keep masks of a training block (attention branch, then MLP branch,
    the order of the reference's two DropPath calls, models.py:291-294), or None.  timm's drop_path
    on the reference's LND tensor draws ONE value per token position (shape (L, 1, 1)), shared by
    every image of the batch, and divides by the keep probability."""
    dpm = blk.drop_path
    if not isinstance(dpm, DropPath) or not dpm.drop_prob:
        return None
    keep = 1.0 - dpm.drop_prob
    ms = []
    for _ in range(2):
        m = torch.empty(ntok, dtype=torch.float32, device=device).bernoulli_(keep)
        if keep > 0.0:
            m.div_(keep)
        ms.append(m)
    return tuple(ms)


class CLIPResNet(nn.Module):
    """Importable for API compatibility; ResNet backbones are outside the ViT hot path."""

    def __init__(self, *args, **kwargs):
        super().__init__()
        raise NotImplementedError("CLIPResNet is out of scope of the MI355X ViT build (SURVEY §2 row 8)")


class CLIPResNetWithAttention(CLIPResNet):
    pass


# ============================================================================ text path
class CLIPTextEncoder(nn.Module):
    """Reference models.py:600-714 (plain torch; batch-independent and frozen)."""

    def __init__(self, context_length=77, vocab_size=49408, transformer_width=512, transformer_heads=8,
                 transformer_layers=12, embed_dim=512, pretrained=None, **kwargs):
        super().__init__()
        self.pretrained = pretrained
        self.context_length = context_length
        self.transformer = Transformer(transformer_width, transformer_layers, transformer_heads,
                                       attn_mask=self.build_attention_mask())
        self.vocab_size = vocab_size
        self.token_embedding = nn.Embedding(vocab_size, transformer_width)
        self.positional_embedding = nn.Parameter(torch.empty(context_length, transformer_width))
        self.ln_final = LayerNorm(transformer_width)
        self.text_projection = nn.Parameter(torch.empty(transformer_width, embed_dim))
        self._output_dim = embed_dim
        self.apply(self._init_weights_default)
        nn.init.normal_(self.positional_embedding, std=0.01)
        nn.init.normal_(self.text_projection, std=transformer_width ** -0.5)

    def _init_weights_default(self, m):
        if isinstance(m, nn.Linear):
            nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, std=0.02)

    def build_attention_mask(self):
        return torch.full((self.context_length, self.context_length), float("-inf")).triu_(1)

    def forward(self, text):
        x = self.token_embedding(text)
        pos = self.positional_embedding[: x.shape[1]]
        x = (x + pos.to(x.dtype)).permute(1, 0, 2)
        x = self.transformer(x).permute(1, 0, 2)
        x = self.ln_final(x)
        return x[torch.arange(x.shape[0], device=x.device), text.argmax(dim=-1)] @ self.text_projection


class CLIPTextContextEncoder(nn.Module):
    """Reference models.py:785-864: class tokens with learnable context tokens inserted after
    SOT, causal mask, EOT read-out.  Plain torch."""

    def __init__(self, context_length=22, vocab_size=49408, transformer_width=512, transformer_heads=8,
                 transformer_layers=12, embed_dim=512, out_dim=256, pretrained=None, **kwargs):
        super().__init__()
        self.pretrained = pretrained
        self.context_length = context_length
        self.transformer = Transformer(transformer_width, transformer_layers, transformer_heads,
                                       attn_mask=self.build_attention_mask())
        self.embed_dim = embed_dim
        self.vocab_size = vocab_size
        self.token_embedding = nn.Embedding(vocab_size, transformer_width)
        self.positional_embedding = nn.Parameter(torch.empty(context_length, transformer_width))
        self.ln_final = LayerNorm(transformer_width)
        self.text_projection = nn.Parameter(torch.empty(transformer_width, embed_dim))
        # the reference leaves these two as uninitialised torch.empty (models.py:811,813);
        # give them defined values so an un-loaded model is finite
        nn.init.normal_(self.positional_embedding, std=0.01)
        nn.init.normal_(self.text_projection, std=transformer_width ** -0.5)

    def init_weights(self, pretrained=None):
        pretrained = pretrained or self.pretrained
        if not isinstance(pretrained, str):
            return
        ckpt = torch.jit.load(pretrained, map_location="cpu").float().state_dict()
        sd = {}
        for k, v in ckpt.items():
            if k.startswith("transformer.") or k.startswith("token_embedding") or k.startswith("ln_final") \
                    or k in ("positional_embedding", "text_projection"):
                if k == "positional_embedding" and v.shape[0] > self.context_length:
                    v = v[: self.context_length]
                sd[k] = v
        self.load_state_dict(sd, strict=False)

    def build_attention_mask(self):
        return torch.full((self.context_length, self.context_length), float("-inf")).triu_(1)

    def forward(self, text, context):
        x_text = self.token_embedding(text)
        K, N1, C = x_text.shape
        B, N2, _ = context.shape
        eos = (text.argmax(dim=-1) + N2).reshape(1, K).expand(B, K).reshape(-1)
        x_text = x_text.reshape(1, K, N1, C).expand(B, K, N1, C)
        context = context.reshape(B, 1, N2, C).expand(B, K, N2, C)
        x = torch.cat([x_text[:, :, 0:1], context, x_text[:, :, 1:]], dim=2).reshape(B * K, N1 + N2, C)
        x = (x + self.positional_embedding).permute(1, 0, 2)
        x = self.transformer(x).permute(1, 0, 2)
        x = self.ln_final(x)
        x = x[torch.arange(x.shape[0], device=x.device), eos] @ self.text_projection
        return x.reshape(B, K, self.embed_dim)


# ============================================================================ neck
class ViTFeatureFusionNeck(nn.Module):
    """Reference models.py:717-782: per-level 3x3 ConvBNReLU, concat, 1x1 ConvBNReLU."""

    def __init__(self, in_channels_list, out_channels, inter_channels=None):
        super().__init__()
        if not isinstance(in_channels_list, (list, tuple)):
            raise TypeError("in_channels_list must be a list or tuple")
        inter_channels = inter_channels or out_channels
        self.num_inputs = len(in_channels_list)
        self.process_layers = nn.ModuleList(
            [ConvBNReLU(c, inter_channels, kernel_size=3, padding=1) for c in in_channels_list])
        self.fusion_layer = ConvBNReLU(inter_channels * self.num_inputs, out_channels, kernel_size=1, padding=0)
        self.apply(self._init_weights)

    def _init_weights(self, m):
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)

    @staticmethod
    def _conv_bn_relu(layer, x):
        """ConvBNReLU with the conv on the MFMA implicit-GEMM kernels for 16-bit maps where
        the shape allows (3x3: Cin % 128 == 0; 1x1: Cin, Cout % 64 == 0), BN (batch
        statistics in train mode) and ReLU on the channels-last result.  fp32 maps (fp32
        images) keep fp32 convs, the reference's arithmetic."""
        conv, bn, act = layer[0], layer[1], layer[2]
        if x.dtype in (torch.bfloat16, torch.float16) and conv.kernel_size == (3, 3) \
                and ops.conv3x3_supported(x, conv.weight):
            y = ops.Conv3x3Fn.apply(x, conv.weight, x.dtype)
        elif x.dtype in (torch.bfloat16, torch.float16) and conv.kernel_size == (1, 1) \
                and ops.conv1x1_supported(x, conv.weight):
            y = ops.Conv1x1Fn.apply(x, conv.weight, conv.bias, x.dtype)
        else:
            ops.note_torch_fallback()
            y = conv(x)
        if ops.bn_hip_ok(bn, y):
            return ops.bn_train(bn, y, relu=True)  # BN + ReLU in one pass each way
        if ops.bn_eval_ok(bn, y):
            return ops.bn_eval(bn, y, relu=True)   # eval: running statistics, ReLU fused
        ops.note_torch_fallback()
        return act(bn(y))

    def forward(self, features):
        if len(features) != self.num_inputs:
            raise ValueError(f"ViTFeatureFusionNeck got {len(features)} inputs, expected {self.num_inputs}")
        if not features[0].is_cuda:
            feats = [layer(f) for layer, f in zip(self.process_layers, features)]
            return [self.fusion_layer(torch.cat(feats, dim=1))]
        if ops.neck_levels_hip_ok(self.process_layers, features):
            # train mode: the 12 ConvModules write their slices of one concatenated buffer
            # (no torch.cat), BN + ReLU fused (ops.NeckLevelsFn)
            layers = list(self.process_layers)
            cat = ops.NeckLevelsFn.apply((tuple(layer[1] for layer in layers), features[0].dtype), *features,
                                         *[layer[0].weight for layer in layers], *[layer[1].weight for layer in layers],
                                         *[layer[1].bias for layer in layers])
        else:
            feats = [self._conv_bn_relu(layer, f) for layer, f in zip(self.process_layers, features)]
            cat = torch.cat(feats, dim=1)  # channels-last in, channels-last out
        return [self._conv_bn_relu(self.fusion_layer, cat)]


# ============================================================================ context decoder
class Attention(nn.Module):
    """Reference models.py:311-344."""

    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_scale=None, attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.num_heads = num_heads
        self.scale = qk_scale or (dim // num_heads) ** -0.5
        self.q_proj = nn.Linear(dim, dim, bias=qkv_bias)
        self.k_proj = nn.Linear(dim, dim, bias=qkv_bias)
        self.v_proj = nn.Linear(dim, dim, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)

    def forward(self, q, k, v):
        B, Nq, C = q.shape
        Mk = k.shape[1]
        h = self.num_heads
        q = self.q_proj(q).reshape(B, Nq, h, C // h)
        k = self.k_proj(k).reshape(B, Mk, h, C // h)
        v = self.v_proj(v).reshape(B, Mk, h, C // h)
        attn = (torch.einsum("bnkc,bmkc->bknm", q, k) * self.scale).softmax(dim=-1)
        x = torch.einsum("bknm,bmkc->bnkc", attn, v).reshape(B, Nq, C)
        return self.proj_drop(self.proj(x))


class TransformerDecoderLayer(nn.Module):
    """Reference models.py:346-375."""

    def __init__(self, d_model, nhead, dropout=0.1):
        super().__init__()
        self.self_attn = Attention(d_model, nhead, proj_drop=dropout)
        self.cross_attn = Attention(d_model, nhead, proj_drop=dropout)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.norm3 = nn.LayerNorm(d_model)
        self.dropout = nn.Dropout(dropout)
        self.mlp = nn.Sequential(nn.Linear(d_model, d_model * 4), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(d_model * 4, d_model))

    def forward(self, x, mem):
        q = k = v = self.norm1(x)
        x = x + self.self_attn(q, k, v)
        q = self.norm2(x)
        x = x + self.cross_attn(q, mem, mem)
        return x + self.dropout(self.mlp(self.norm3(x)))


class ContextDecoder(nn.Module):
    """Reference models.py:867-917 (text queries cross-attend over the visual context)."""

    def __init__(self, transformer_width=256, transformer_heads=4, transformer_layers=6, visual_dim=1024,
                 dropout=0.1, **kwargs):
        super().__init__()
        self.memory_proj = nn.Sequential(nn.LayerNorm(visual_dim), nn.Linear(visual_dim, transformer_width),
                                         nn.LayerNorm(transformer_width))
        self.text_proj = nn.Sequential(nn.LayerNorm(visual_dim), nn.Linear(visual_dim, transformer_width))
        self.decoder = nn.ModuleList([TransformerDecoderLayer(transformer_width, transformer_heads, dropout)
                                      for _ in range(transformer_layers)])
        self.out_proj = nn.Sequential(nn.LayerNorm(transformer_width), nn.Linear(transformer_width, visual_dim))
        self.apply(self._init_weights)

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def forward(self, text, visual):
        visual = self.memory_proj(visual)
        x = self.text_proj(text)
        for layer in self.decoder:
            x = layer(x, visual)
        return self.out_proj(x)
