"""DenseCLIP segmentor (reference seg/denseclip/denseclip.py:60-1087), same constructor and
forward contract, built on the HIP ViT backbone.

Differences from the reference, all deliberate:
  * errors RAISE (the reference catches everything in forward and returns None outputs,
    denseclip.py:733-752, which hides kernel failures);
  * no defensive `.clone()` of the 12 feature maps (denseclip.py:586, 743);
  * the score map (denseclip.py:670-675) is computed on the HIP kernels from the token buffer
    behind the last map (read in place): the pooling as a strided row mean, vis_proj as an MFMA
    GEMM and the normalise-and-contract as a batched [K x C] . [C x pixels] MFMA product.  It is returned by `_process_features` and, exactly as
    in the reference, not used by the heads (denseclip.py:747);
  * the final logits/depth resize is the HIP bilinear kernel (fp32 output).
"""
import logging
from collections import OrderedDict

import torch
import torch.nn as nn

from . import ops
from .heads import FCNHead, IdentityHead
from .models import (CLIPResNet, CLIPResNetWithAttention, CLIPTextContextEncoder, CLIPTextEncoder,
                     CLIPVisionTransformer, ContextDecoder, ViTFeatureFusionNeck)
from .utils import tokenize

logger = logging.getLogger(__name__)


class DenseCLIP(nn.Module):
    def __init__(self, backbone, text_encoder, decode_head, class_names, context_length, depth_head=None,
                 context_decoder=None, neck=None, context_feature="attention", score_concat_index=3,
                 text_head=False, tau=0.07, auxiliary_head=None, identity_head=None, train_cfg=None,
                 test_cfg=None, token_embed_dim=512, text_dim=512, clip_pretrained_path=None, **kwargs):
        super().__init__()
        self.class_names = class_names
        self.num_classes = len(class_names)
        self.fixed_text_context_length = context_length
        self.context_feature = context_feature
        self.score_concat_index = score_concat_index
        self.text_head = text_head
        self.tau = tau
        self.train_cfg = train_cfg
        self.test_cfg = test_cfg
        self.align_corners = False
        self.text_dim = text_dim
        # True: the train-mode forward returns the heads' low-res outputs and train.loss_fn
        # evaluates upsample + CE / SILog in fused kernels (ops.UpsampleCEFn / UpsampleSILogFn).
        # False (default): the reference contract — upsampled 'main_output' / 'depth_output'.
        self.fused_head_loss = False
        self.graph_text = True  # replay the frozen text path from a HIP graph (see _text_embeddings)
        # fp32 images (the reference trainer's input): run the neck and heads on the HIP kernels in
        # the backbone's 16-bit compute dtype (outputs returned in fp32) whenever their widths
        # allow it (ops.neck_heads_hip_capable); False keeps them in fp32 torch (for A/B tests)
        self.hip_heads = True

        # ---- backbone (denseclip.py:111-126)
        bcfg = dict(backbone)
        btype = bcfg.pop("type")
        if btype == "CLIPVisionTransformer":
            self.backbone = CLIPVisionTransformer(**bcfg)
            backbone_out = backbone.get("width", 768)
        elif btype == "CLIPResNet":
            self.backbone = CLIPResNet(**bcfg)
        elif btype == "CLIPResNetWithAttention":
            self.backbone = CLIPResNetWithAttention(**bcfg)
        else:
            raise ValueError(f"Unsupported backbone type: {btype}")

        # ---- text encoder (denseclip.py:130-152)
        tcfg = dict(text_encoder)
        ttype = tcfg.pop("type")
        enc_dim = text_encoder.get("embed_dim")
        if enc_dim is not None and enc_dim != self.text_dim:
            self.text_dim = enc_dim
        tcfg["embed_dim"] = self.text_dim
        self.is_context_encoder = False
        if ttype == "CLIPTextEncoder":
            tcfg["context_length"] = self.fixed_text_context_length
            self.text_encoder = CLIPTextEncoder(**tcfg)
        elif ttype == "CLIPTextContextEncoder":
            if text_encoder.get("context_length") is None:
                raise ValueError("`context_length` required in CLIPTextContextEncoder config.")
            self.text_encoder = CLIPTextContextEncoder(**tcfg)
            self.is_context_encoder = True
        else:
            raise ValueError(f"Unsupported text_encoder type: {ttype}")

        if clip_pretrained_path:
            self._load_clip(clip_pretrained_path)

        # ---- projections (denseclip.py:195-200)
        self.vis_proj = None
        self.global_proj = None
        if backbone_out != self.text_dim:
            self.vis_proj = nn.Conv2d(backbone_out, self.text_dim, kernel_size=1)
            self.global_proj = nn.Linear(backbone_out, self.text_dim)

        # ---- context decoder (denseclip.py:204-211)
        self.context_decoder = None
        if context_decoder:
            ccfg = dict(context_decoder)
            if ccfg.pop("type") != "ContextDecoder":
                raise ValueError("Unsupported context decoder type")
            ccfg["visual_dim"] = self.text_dim
            self.context_decoder = ContextDecoder(**ccfg)

        # ---- neck (denseclip.py:214-287)
        self.neck = None
        head_in = backbone_out
        if neck:
            ntype = neck.get("type")
            if ntype == "ViTFeatureFusionNeck":
                outs = backbone.get("out_indices", [])
                if not outs:
                    raise ValueError("Backbone config must specify 'out_indices' when using ViTFeatureFusionNeck.")
                out_ch = neck.get("out_channels")
                if not isinstance(out_ch, int) or out_ch <= 0:
                    raise ValueError("Neck config for 'ViTFeatureFusionNeck' requires a positive 'out_channels'.")
                self.neck = ViTFeatureFusionNeck([backbone.get("width", 768)] * len(outs), out_ch,
                                                 neck.get("inter_channels"))
                head_in = out_ch
            elif ntype == "FPN":
                raise NotImplementedError("FPN neck (ResNet configs) is outside the ViT build")
            else:
                raise ValueError(f"Unsupported neck type: {ntype}")

        # ---- decode head (denseclip.py:290-323)
        self.decode_head = None
        if decode_head:
            dtype_ = decode_head.get("type")
            self.align_corners = decode_head.get("align_corners", False)
            if self.align_corners:
                # the resize kernels (bilinear, fused resize + CE / SILog) implement the
                # config's align_corners=False only (denseclip.py:847, 860, 899, 909)
                raise NotImplementedError("decode_head.align_corners=True is not supported by the HIP resize kernels")
            self.num_classes = decode_head.get("num_classes", self.num_classes)
            hin = decode_head.get("in_channels", head_in)
            if dtype_ == "FPNHead":
                ch = decode_head.get("channels", 256)
                self.decode_head = FCNHead(hin, ch)
                self.decode_head.classifier = nn.Conv2d(ch, self.num_classes, kernel_size=1)
            elif dtype_ == "IdentityHead":
                self.decode_head = IdentityHead()
            else:
                raise ValueError(f"Unsupported/unavailable decode_head type: {dtype_}")
        self.with_decode_head = self.decode_head is not None

        # ---- depth head (denseclip.py:327-357)
        self.depth_head = None
        self.with_depth_head = False
        if depth_head:
            if depth_head.get("align_corners", False):
                raise NotImplementedError("depth_head.align_corners=True is not supported by the HIP resize kernels")
            if depth_head.get("type") == "FCNHeadDepth":
                ch = depth_head.get("channels", 128)
                self.depth_head = FCNHead(depth_head.get("in_channels", head_in), ch)
                self.depth_head.classifier = nn.Conv2d(ch, 1, kernel_size=1)
                self.with_depth_head = True
            else:
                logger.warning(f"Unsupported depth_head type: {depth_head.get('type')}")

        self.auxiliary_head = None
        self.with_auxiliary_head = False
        self.identity_head = None
        self.with_identity_head = False

        # ---- class-name tokens + learnable context (denseclip.py:373-408)
        self.texts = torch.cat([tokenize(c, context_length=self.fixed_text_context_length) for c in class_names])
        self.contexts = None
        self.gamma = None
        if self.is_context_encoder:
            n_ctx = getattr(self.text_encoder, "context_length", 77) - self.fixed_text_context_length
            if n_ctx > 0:
                self.contexts = nn.Parameter(torch.randn(1, n_ctx, token_embed_dim))
                nn.init.trunc_normal_(self.contexts, std=0.02)
            self.gamma = nn.Parameter(torch.ones(self.text_dim) * 1e-4)
        self._init_non_clip_weights()

    # ------------------------------------------------------------------ init / loading
    def _load_clip(self, path):
        """OpenAI CLIP TorchScript checkpoint -> backbone (visual.*) + text encoder
        (denseclip.py:156-191).  A missing file is logged, as in the reference."""
        try:
            sd = torch.jit.load(path, map_location="cpu").state_dict()
        except (FileNotFoundError, ValueError, RuntimeError) as e:
            logger.error(f"Error loading CLIP weights from {path}: {e}")
            return
        vis = OrderedDict((k[7:], v) for k, v in sd.items() if k.startswith("visual."))
        if vis:
            self.backbone.load_state_dict(vis, strict=False)
        txt = OrderedDict()
        prefixes = ("transformer.", "token_embedding.", "positional_embedding", "ln_final.", "text_projection")
        for k, v in sd.items():
            if not k.startswith(prefixes):
                continue
            if k == "positional_embedding":
                n = self.text_encoder.positional_embedding.shape[0]
                if v.shape[0] >= n:
                    txt[k] = v[:n]
            elif k == "text_projection":
                if v.shape == self.text_encoder.text_projection.shape:
                    txt[k] = v
            else:
                txt[k] = v
        if txt:
            self.text_encoder.load_state_dict(txt, strict=False)

    def _init_weights_fn(self, m):
        name = m.__class__.__name__
        if "Conv" in name and hasattr(m, "weight"):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif "Linear" in name:
            nn.init.normal_(m.weight, 0, 0.01)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif "BatchNorm" in name or "GroupNorm" in name:
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)

    def _init_non_clip_weights(self):
        """denseclip.py:448-513."""
        for name in ("vis_proj", "global_proj", "context_decoder", "neck", "decode_head", "depth_head"):
            mod = getattr(self, name)
            if mod is None:
                continue
            mod.apply(self._init_weights_fn)
            if name in ("decode_head", "depth_head") and isinstance(getattr(mod, "classifier", None), nn.Conv2d):
                nn.init.normal_(mod.classifier.weight, mean=0, std=0.01)
                if mod.classifier.bias is not None:
                    nn.init.constant_(mod.classifier.bias, 0)

    # ------------------------------------------------------------------ forward pieces
    def extract_feat(self, img):
        feats = self.backbone(img)
        if not isinstance(feats, (list, tuple)) or not feats:
            raise RuntimeError("backbone returned no feature maps")
        return list(feats)

    def _text_forward(self, texts):
        if isinstance(self.text_encoder, CLIPTextContextEncoder) and self.contexts is not None:
            return self.text_encoder(texts, self.contexts)
        return self.text_encoder(texts)

    def _text_prelaunch(self, device):
        """Replay the captured text graph on a side stream at the START of the forward, so its
        ~650 small kernels (a few workgroups each, ~7 ms of a mostly idle GPU when run in line)
        overlap the backbone instead of running between it and the heads; _text_embeddings
        then only waits for it (the score branch runs it under no_grad, so the graph is the path
        either way; the replay reads the parameters' values after the previous optimizer step,
        as an in-line replay would).  A no-op until the graph exists (the first call captures
        it in line) or when a text buffer was re-allocated since the capture."""
        if self.graph_text == "side":  # serve.CapturedForward: the text path eager on the side stream, captured
            self._text_side_eager(device)
            return
        g = getattr(self, "_text_graph", None)
        if g is None or not self.graph_text:
            return
        device = torch.device(device)
        if device.type != "cuda":
            return
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        params = list(self.text_encoder.parameters())
        if self.contexts is not None:
            params.append(self.contexts)
        texts = getattr(self, "_texts_dev", None)
        if texts is None or texts.device != device:
            return
        key = (device, texts.data_ptr(), tuple(p.data_ptr() for p in params), torch.is_autocast_enabled())
        if g[0] != key:
            return
        main = torch.cuda.current_stream(device)
        side = getattr(self, "_text_stream", None)
        if side is None or side.device != device:
            side = self._text_stream = torch.cuda.Stream(device=device)
        side.wait_stream(main)  # after every earlier use of the graph's output buffer
        with torch.cuda.stream(side):
            g[1].replay()
        self._text_pending = (key, side)

    def _text_side_eager(self, device):
        """graph_text == "side" (set while serve.CapturedForward captures the forward): launch the text
        path eagerly on the side stream, forked from the main stream and joined in _text_embeddings —
        inside a stream capture this becomes a parallel branch of the captured graph, so a replay runs
        the text kernels beside the backbone as _text_prelaunch's graph replay does in eager mode."""
        device = torch.device(device)
        if device.type != "cuda":
            return
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        if getattr(self, "_texts_dev", None) is None or self._texts_dev.device != device:
            self._texts_dev = self.texts.to(device)
        main = torch.cuda.current_stream(device)
        side = getattr(self, "_text_stream", None)
        if side is None or side.device != device:
            side = self._text_stream = torch.cuda.Stream(device=device)
        side.wait_stream(main)
        with torch.cuda.stream(side), torch.no_grad():
            out = self._text_forward(self._texts_dev)
        self._text_side_out = (out, side)

    def _text_embeddings(self, B, device):
        """Class-name embeddings (denseclip.py:627-640).  The text path is batch-independent and,
        when frozen (the reference regime and the full fine-tune both freeze it,
        train_denseclip.py:1040-1044), a fixed chain of ~400 small kernels: on a GPU it is
        captured once into a HIP graph and REPLAYED every step (recomputed, not cached), which
        removes the per-kernel launch gaps; any trainable text parameter, or a parameter
        re-allocated since the capture, falls back to eager execution / a new capture."""
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            # "cuda" and "cuda:0" compare unequal: without this the token ids were re-uploaded on
            # every call, freeing the tensor a captured graph reads (a replay then gathered
            # through a recycled block: test_text_path_graph_replay_matches_eager faulted)
            device = torch.device("cuda", torch.cuda.current_device())
        if getattr(self, "_texts_dev", None) is None or self._texts_dev.device != device:
            self._texts_dev = self.texts.to(device)
        texts = self._texts_dev
        params = list(self.text_encoder.parameters())
        if self.contexts is not None:
            params.append(self.contexts)
        # no autograd graph is recorded when gradients are off (the score-map branch runs under
        # no_grad: its output is discarded, denseclip.py:747), trainable parameters or not
        frozen = not torch.is_grad_enabled() or not any(p.requires_grad for p in params)
        side_out = getattr(self, "_text_side_out", None)
        self._text_side_out = None
        if side_out is not None:  # launched by _text_side_eager at the start of this forward
            torch.cuda.current_stream(device).wait_stream(side_out[1])
            return side_out[0].expand(B, -1, -1)
        if not (self.graph_text and frozen and device.type == "cuda"):
            return self._text_forward(texts).expand(B, -1, -1)
        # every device buffer the graph reads is in the key: a re-allocated one forces a new capture
        key = (device, texts.data_ptr(), tuple(p.data_ptr() for p in params), torch.is_autocast_enabled())
        g = getattr(self, "_text_graph", None)
        pend = getattr(self, "_text_pending", None)
        self._text_pending = None
        if pend is not None and g is not None and pend[0] == key == g[0]:
            torch.cuda.current_stream(device).wait_stream(pend[1])  # replayed by _text_prelaunch
            return g[2].expand(B, -1, -1)
        if g is None or g[0] != key:
            side = torch.cuda.Stream(device=device)
            side.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(side), torch.no_grad():
                self._text_forward(texts)  # warm-up outside the capture (allocator, library handles)
            torch.cuda.current_stream(device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            # thread-local capture: other threads' HIP calls (RCCL / DDP helpers) stay legal
            with torch.no_grad(), torch.cuda.graph(graph, capture_error_mode="thread_local"):
                out = self._text_forward(texts)
            self._text_graph = g = (key, graph, out)
        g[1].replay()
        return g[2].expand(B, -1, -1)

    def _process_features(self, x):
        """Global feature, projections, text embeddings, context fusion and the pixel-text
        score map (denseclip.py:570-698).  Returns (text, features_for_head, score, x)."""
        if not isinstance(x, (list, tuple)) or not x:
            raise ValueError("expected a non-empty list of feature maps")
        visual = x[-1]
        if visual.ndim != 4:
            raise ValueError(f"Expected last backbone feature map to be 4D, got {visual.ndim}D")
        B, Cv, h, w = visual.shape
        HW = h * w
        cdt = visual.dtype if visual.dtype in (torch.bfloat16, torch.float16) else \
            getattr(self.backbone, "compute_dtype", torch.float16)
        # the score branch is forward-only, as in the reference: with score_concat_index >= 0 the
        # reference concatenates the score map onto a CLONE of the maps and the forward passes
        # the unmodified maps to the neck (denseclip.py:586, 684-694, 747), so nothing trainable
        # is reached through it (its parameters are kept out of DDP: train.gradless_parameter_names)
        with torch.no_grad():
            # pixel rows of the last map read in place: the read-out map is a channels-last view
            # of a (B*N, C) token buffer (CLS rows in between, ops.ReadoutFn), so the pooling, the
            # vis_proj GEMM and the score map run on that buffer with a batch stride and a row
            # offset — no NHWC copy of the map.  Any other map layout gets one NHWC copy.
            tok = ops.token_rows(visual)
            if tok is not None and tok.dtype == cdt:
                rows, Nr, off = tok, HW + 1, 1
            else:
                rows, Nr, off = visual.permute(0, 2, 3, 1).reshape(B * HW, Cv).to(cdt).contiguous(), HW, 0
            g = ops.row_mean(rows, B, HW, row_off=off, bstride=Nr * Cv)    # adaptive_avg_pool2d
            if self.global_proj is not None:
                g = ops.gemm(ops.cast(g, cdt), ops.WEIGHTS.get(self.global_proj.weight, cdt),
                             bias=self.global_proj.bias.detach(), out_dtype=torch.float32)
            if self.vis_proj is not None:  # 1x1 conv over every row (the B CLS rows ride along)
                v = ops.gemm(rows, ops.WEIGHTS.get(self.vis_proj.weight, cdt), bias=self.vis_proj.bias.detach())
            else:
                v = rows
            Ct = v.shape[1]
            text = self._text_embeddings(B, visual.device)
            if self.context_decoder is not None:
                vpix = v.view(B, Nr, Ct)[:, off:].float()
                if self.context_feature == "attention":
                    ctx = torch.cat([g.unsqueeze(1), vpix], dim=1)
                elif self.context_feature == "backbone":
                    ctx = vpix
                else:
                    raise ValueError(f"Invalid context_feature type: {self.context_feature}")
                text = text + self.gamma * self.context_decoder(text, ctx)
            if Ct != text.shape[2]:
                raise ValueError(f"Visual dim after proj ({Ct}) != Text dim ({text.shape[2]}).")
            score = ops.score_map(v, text, B, HW, row_off=off, bstride=Nr * Ct).view(B, -1, h, w)
        feats = list(x)
        if 0 <= self.score_concat_index < len(feats):
            with torch.no_grad():  # one pass: copy + resize into the concatenated map
                feats[self.score_concat_index] = ops.score_concat(feats[self.score_concat_index], score)
        return text, feats, score, list(x)

    def _heads(self, x_maps):
        if self.neck is not None:
            fused = self.neck(x_maps)
            inp = fused[0] if isinstance(fused, (list, tuple)) else fused
        else:
            inp = x_maps[-1]
        seg = self.decode_head(inp) if self.with_decode_head else None
        depth = self.depth_head(inp) if self.with_depth_head else None
        return seg, depth

    def _hip_heads_dtype(self, img):
        """The 16-bit dtype the neck / heads run in for this input on the fp32-image path, or None
        (16-bit images already give 16-bit maps; CPU tensors, fp32 compute or widths without a HIP
        kernel keep the fp32 torch neck / heads)."""
        if not (self.hip_heads and img.is_cuda and img.dtype == torch.float32
                and isinstance(self.backbone, CLIPVisionTransformer)):
            return None
        cdt = self.backbone.compute_dtype
        if cdt not in (torch.float16, torch.bfloat16) or not ops.neck_heads_hip_capable(self):
            return None
        return cdt

    def _forward_hip_heads(self, img, cdt):
        """fp32 images with the neck and heads on the HIP kernels: the backbone returns its maps in
        the compute dtype (channels-last token-buffer views the implicit-GEMM convs read in place),
        the neck / heads run in it, and their low-res outputs come back in fp32 through
        ops.HeadsOutFn (whose backward applies the fp16 gradient scale, ops.HeadScale)."""
        hs = ops.HeadScale(img.device, cdt)
        with ops.head_scale(hs):
            feats = self.backbone(img, map_dtype=cdt)
            if not isinstance(feats, (list, tuple)) or not feats:
                raise RuntimeError("backbone returned no feature maps")
            feats = list(feats)
            self._process_features(feats)  # score branch: computed and discarded (denseclip.py:747)
            with torch.autocast("cuda", dtype=cdt):
                seg, depth = self._heads(feats)
        outs = [t for t in (seg, depth) if t is not None]
        res = list(ops.HeadsOutFn.apply(hs, *outs)) if outs else []
        seg = res.pop(0) if seg is not None else None
        depth = res.pop(0) if depth is not None else None
        return seg, depth

    def forward(self, img, img_metas=None, gt_semantic_seg=None, return_loss=True, **kwargs):
        """denseclip.py:702-916.  Train: {'main_output','depth_output','aux_losses'};
        eval: {'seg','depth'} resized to the image."""
        if img.is_cuda:
            self._text_prelaunch(img.device)
        hcdt = self._hip_heads_dtype(img)
        if hcdt is not None:
            seg, depth = self._forward_hip_heads(img, hcdt)
        else:
            feats = self.extract_feat(img)
            self._process_features(feats)  # score branch: computed and discarded (denseclip.py:747)
            maps = feats
            param = next(self.neck.parameters()) if self.neck is not None else None
            if param is not None and maps[0].dtype != param.dtype and maps[0].is_cuda:
                with torch.autocast("cuda", dtype=maps[0].dtype):
                    seg, depth = self._heads(maps)
            else:
                seg, depth = self._heads(maps)
        if return_loss and self.training and self.fused_head_loss:
            # low-res head outputs for train.loss_fn's fused upsample + CE / SILog kernels
            # (same loss and gradients; the 1024x2048 logits are never materialised)
            return {"main_output": None, "depth_output": None, "aux_losses": {},
                    "main_output_lowres": seg, "depth_output_lowres": depth}
        if return_loss and self.training:
            gt = None
            for cand in (gt_semantic_seg, kwargs.get("gt_depth"), kwargs.get("depth_targets"),
                         kwargs.get("seg_targets")):
                if cand is not None:
                    gt = tuple(cand.shape[-2:])
                    break
            if seg is not None and gt is not None and tuple(seg.shape[-2:]) != gt:
                seg = ops.upsample(seg, gt)
            if depth is not None and gt is not None and tuple(depth.shape[-2:]) != gt:
                depth = ops.upsample(depth, gt)
            return {"main_output": seg, "depth_output": depth, "aux_losses": {}}
        hw = tuple(img.shape[2:])
        if seg is not None and tuple(seg.shape[-2:]) != hw:
            seg = ops.upsample(seg, hw)
        if depth is not None and tuple(depth.shape[-2:]) != hw:
            depth = ops.upsample(depth, hw)
        return {"seg": seg, "depth": depth}

    def inference(self, img, img_meta, rescale):
        out = self.forward(img, img_metas=img_meta, return_loss=False)
        seg, depth = out.get("seg"), out.get("depth")
        if rescale and img_meta and "ori_shape" in img_meta[0]:
            shp = tuple(img_meta[0]["ori_shape"][:2])
            if seg is not None and tuple(seg.shape[-2:]) != shp:
                seg = ops.upsample(seg, shp)
            if depth is not None and tuple(depth.shape[-2:]) != shp:
                depth = ops.upsample(depth, shp)
        return {"seg": seg, "depth": depth}

    def simple_test(self, img, img_meta, rescale=True):
        out = self.inference(img, img_meta, rescale)
        seg = out["seg"].argmax(dim=1).cpu().numpy()[0] if out["seg"] is not None else None
        depth = out["depth"].squeeze(1).cpu().numpy()[0] if out["depth"] is not None else None
        return {"seg": seg, "depth": depth}

    def aug_test(self, imgs, img_metas, rescale=True):
        segs, depths = [], []
        for img, meta in zip(imgs, img_metas):
            out = self.inference(img.unsqueeze(0), [meta], rescale)
            if out["seg"] is not None:
                segs.append(out["seg"])
            if out["depth"] is not None:
                depths.append(out["depth"])
        seg = torch.stack(segs).mean(0).argmax(dim=1).squeeze(0).cpu().numpy() if segs else None
        depth = torch.stack(depths).mean(0).squeeze().cpu().numpy() if depths else None
        return {"seg": seg, "depth": depth}

    def forward_dummy(self, img):
        seg, _ = self._heads(self.extract_feat(img))
        return seg
