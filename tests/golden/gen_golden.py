"""Generate golden fixtures by running the REFERENCE DenseCLIP on CPU (fp32).

Run ONLY in the development container (the reference tree does not travel to the
GPU box):

    python tests/golden/gen_golden.py            # writes tests/golden/*.safetensors
    python tests/golden/gen_golden.py ctx        # only the ContextDecoder fixture (+ manifest)
    python tests/golden/gen_golden.py vitl14     # only the ViT-L/14 fixture (+ manifest)
    python tests/golden/gen_golden.py mid        # only the MID_CFG fixtures (+ manifest)
    python tests/golden/gen_golden.py full8193   # only the 1x1024x2048 (N = 8193) ViT-B/16 fixture

The reference package imports `timm`, `ftfy` and `torchvision`, none of which are
installed here.  The shims below are written into a temporary directory at run
time (never into the repo's product package).  They only cover names the ViT path
does not compute with:
  * timm.layers.drop_path / drop  -> identity at drop_path_rate 0 (models.py:265)
  * timm.layers.trunc_normal_     -> torch.nn.init.trunc_normal_ (init only; every
                                     weight is overwritten by weights_spec anyway)
  * timm.models.vision_transformer.VisionTransformer -> unused name
  * ftfy.fix_text                 -> identity (class names are plain ASCII)
  * torchvision FCNHead           -> torchvision's published definition
        Sequential(Conv2d(in, in//4, 3, pad 1, bias=False), BatchNorm2d(in//4),
                   ReLU(), Dropout(0.1), Conv2d(in//4, channels, 1))
    (torchvision is not pinned by the reference; parity at the head boundary is
    pinned only by this restatement — see DESIGN.md "parity".)
  * torchvision FeaturePyramidNetwork / LastLevelMaxPool -> unused stubs.
Every floating-point state-dict entry is then overwritten from weights_spec.py so
the fixture is reproducible in the tests without shipping weights.
"""
import os
import sys
import tempfile
import textwrap

import torch
import torch.nn as nn
import torch.nn.functional as F
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from weights_spec import fill_state_dict  # noqa: E402
from model_configs import (TINY_CFG, TINY_CTX_CFG, CTX_GAMMA, CITYSCAPES_CFG, CITYSCAPES_CLASSES,  # noqa: E402
                           VITL14_CFG, MID_CFG)

REF_SEG = "/root/reference/segmentation"

SHIMS = {
    "timm/__init__.py": "",
    "timm/layers/__init__.py": textwrap.dedent("""
        import torch
        def drop_path(x, drop_prob=0., training=False, scale_by_keep=True):
            if drop_prob == 0. or not training:
                return x
            raise NotImplementedError('shim: drop_path>0 not used by the fixtures')
        def drop(*a, **k):
            raise NotImplementedError
        def trunc_normal_(t, mean=0., std=1., a=-2., b=2.):
            return torch.nn.init.trunc_normal_(t, mean=mean, std=std, a=a, b=b)
    """),
    "timm/models/__init__.py": "",
    "timm/models/vision_transformer.py": "class VisionTransformer: pass\n",
    "ftfy/__init__.py": "def fix_text(t):\n    return t\n",
    "torchvision/__init__.py": "",
    "torchvision/ops/__init__.py": "",
    "torchvision/ops/feature_pyramid_network.py": textwrap.dedent("""
        import torch.nn as nn
        class FeaturePyramidNetwork(nn.Module):
            def __init__(self, *a, **k):
                super().__init__()
        class LastLevelMaxPool(nn.Module):
            pass
    """),
    "torchvision/models/__init__.py": "",
    "torchvision/models/segmentation/__init__.py": "",
    "torchvision/models/segmentation/fcn.py": textwrap.dedent("""
        import torch.nn as nn
        class FCNHead(nn.Sequential):
            def __init__(self, in_channels, channels):
                inter_channels = in_channels // 4
                layers = [
                    nn.Conv2d(in_channels, inter_channels, 3, padding=1, bias=False),
                    nn.BatchNorm2d(inter_channels),
                    nn.ReLU(),
                    nn.Dropout(0.1),
                    nn.Conv2d(inter_channels, channels, 1),
                ]
                super().__init__(*layers)
    """),
}


def install_shims():
    d = tempfile.mkdtemp(prefix="dclip_shims_")
    for rel, src in SHIMS.items():
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(src)
    sys.path.insert(0, d)
    sys.path.insert(0, REF_SEG)


def build_reference(cfg):
    from denseclip import DenseCLIP  # the reference package
    m = dict(cfg)
    model = DenseCLIP(class_names=CITYSCAPES_CLASSES, **m)
    sd = fill_state_dict(model.state_dict(), seed=0)
    model.load_state_dict(sd, strict=True)
    return model


def capture(model):
    """Hooks to grab the backbone maps, score map and pre-upsample head outputs."""
    cap = {}
    model.backbone.register_forward_hook(lambda m, i, o: cap.__setitem__("maps", [t.detach().clone() for t in o]))
    model.decode_head.register_forward_hook(lambda m, i, o: cap.__setitem__("seg_low", o.detach().clone()))
    model.depth_head.register_forward_hook(lambda m, i, o: cap.__setitem__("depth_low", o.detach().clone()))
    orig = model._process_features

    def wrapped(x):
        out = orig(x)
        cap["text"] = out[0].detach().clone()
        cap["score"] = out[2].detach().clone()
        return out
    model._process_features = wrapped
    return cap


def stats(t):
    t = t.double()
    return torch.tensor([t.mean(), t.std(), t.norm(), t.abs().max()], dtype=torch.float64)


def sample_idx(numel, k, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randperm(numel, generator=g)[:k]


def images(b, h, w, seed=1234):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(b, 3, h, w, generator=g)


def train_step_fixture(cfg, b, h, w):
    """One seeded train step of the reference (dropout disabled -> deterministic; BN in train
    mode uses batch statistics, as in the reference trainer): inputs, targets, loss, the
    train-mode low-res head outputs, every gradient's norm and 64 sampled elements."""
    model = build_reference(cfg)
    model.train()
    for mod in model.modules():
        if isinstance(mod, nn.Dropout):
            mod.eval()
    for p in model.parameters():
        p.requires_grad_(True)
    cap = capture(model)
    xb = images(b, h, w, seed=1234)
    g = torch.Generator().manual_seed(1235)
    seg_t = torch.randint(0, 19, (b, h, w), generator=g)
    seg_t[torch.rand(b, h, w, generator=g) < 0.1] = 255
    g = torch.Generator().manual_seed(1236)
    depth_t = 1 + 79 * torch.rand(b, 1, h, w, generator=g)
    depth_m = torch.rand(b, 1, h, w, generator=g) >= 0.2
    out = model(xb, gt_semantic_seg=seg_t, gt_depth=depth_t, return_loss=True)
    sys.path.insert(0, REF_SEG)
    from denseclip.losses import SILogLoss
    ce = F.cross_entropy(out["main_output"], seg_t, ignore_index=255)
    silog = SILogLoss(lambd=0.5, eps=1e-6)(out["depth_output"], depth_t, depth_m)
    loss = 1.0 * ce + 0.1 * silog
    loss.backward()
    tr = {"input": xb, "seg_t": seg_t, "depth_t": depth_t, "depth_m": depth_m.to(torch.uint8),
          "loss": torch.stack([loss.detach(), ce.detach(), silog.detach()]),
          "seg_low": cap["seg_low"], "depth_low": cap["depth_low"]}
    for name, p in model.named_parameters():
        if p.grad is None:
            continue
        gr = p.grad.detach().flatten()
        idx = sample_idx(gr.numel(), min(64, gr.numel()), seed=7)
        tr[f"gnorm/{name}"] = gr.double().norm().reshape(1)
        tr[f"gidx/{name}"] = idx
        tr[f"gval/{name}"] = gr[idx]
    return tr, loss


def gen_mid():
    """MID_CFG (HIP-kernel widths for every neck / head op): an eval forward at 1 x 128x256
    (maps, score map, low-res and resized head outputs) and one train step at 2 x 128x256."""
    model = build_reference(MID_CFG).eval()
    cap = capture(model)
    x = images(1, 128, 256, seed=1234)
    with torch.no_grad():
        out = model(x, return_loss=False)
    t = {"input": x, "seg": out["seg"], "depth": out["depth"], "score": cap["score"],
         "text": cap["text"], "seg_low": cap["seg_low"], "depth_low": cap["depth_low"]}
    for i, mp in enumerate(cap["maps"]):
        t[f"map{i}"] = mp
    save_file({k: v.contiguous() for k, v in t.items()}, os.path.join(HERE, "mid_eval.safetensors"))
    tr, loss = train_step_fixture(MID_CFG, 2, 128, 256)
    save_file({k: v.contiguous() for k, v in tr.items()}, os.path.join(HERE, "mid_train.safetensors"))
    print("mid: loss", loss.item())


def gen_tiny():
    model = build_reference(TINY_CFG).eval()
    cap = capture(model)
    x = images(1, 64, 128, seed=1234)
    with torch.no_grad():
        out = model(x, return_loss=False)
    t = {"input": x, "seg": out["seg"], "depth": out["depth"], "score": cap["score"],
         "text": cap["text"], "seg_low": cap["seg_low"], "depth_low": cap["depth_low"]}
    for i, mp in enumerate(cap["maps"]):
        t[f"map{i}"] = mp
    save_file({k: v.contiguous() for k, v in t.items()}, os.path.join(HERE, "tiny_eval.safetensors"))

    # one seeded train step on the tiny model (dropout disabled -> deterministic;
    # BN in train mode uses batch statistics, as in the reference trainer)
    model = build_reference(TINY_CFG)
    model.train()
    for mod in model.modules():
        if isinstance(mod, nn.Dropout):
            mod.eval()
    for p in model.parameters():
        p.requires_grad_(True)
    xb = images(2, 64, 128, seed=1234)
    g = torch.Generator().manual_seed(1235)
    seg_t = torch.randint(0, 19, (2, 64, 128), generator=g)
    seg_t[torch.rand(2, 64, 128, generator=g) < 0.1] = 255
    g = torch.Generator().manual_seed(1236)
    depth_t = 1 + 79 * torch.rand(2, 1, 64, 128, generator=g)
    depth_m = torch.rand(2, 1, 64, 128, generator=g) >= 0.2
    out = model(xb, gt_semantic_seg=seg_t, gt_depth=depth_t, return_loss=True)
    sys.path.insert(0, REF_SEG)
    from denseclip.losses import SILogLoss
    ce = F.cross_entropy(out["main_output"], seg_t, ignore_index=255)
    silog = SILogLoss(lambd=0.5, eps=1e-6)(out["depth_output"], depth_t, depth_m)
    loss = 1.0 * ce + 0.1 * silog
    loss.backward()
    tr = {"input": xb, "seg_t": seg_t, "depth_t": depth_t, "depth_m": depth_m.to(torch.uint8),
          "loss": torch.stack([loss.detach(), ce.detach(), silog.detach()])}
    for name, p in model.named_parameters():
        if p.grad is None:
            continue
        gr = p.grad.detach().flatten()
        idx = sample_idx(gr.numel(), min(64, gr.numel()), seed=7)
        tr[f"gnorm/{name}"] = gr.double().norm().reshape(1)
        tr[f"gidx/{name}"] = idx
        tr[f"gval/{name}"] = gr[idx]
    save_file({k: v.contiguous() for k, v in tr.items()}, os.path.join(HERE, "tiny_train.safetensors"))
    print("tiny: loss", loss.item())


def gen_tiny_ctx():
    """The tiny model with the ContextDecoder branch, eval: class embeddings after the context
    fusion, the score map and the (unaffected) low-res seg logits."""
    model = build_reference(TINY_CTX_CFG).eval()
    with torch.no_grad():
        model.gamma.fill_(CTX_GAMMA)  # a trained-scale fusion weight, so the branch moves the result
    cap = capture(model)
    x = images(1, 64, 128, seed=1234)
    with torch.no_grad():
        model(x, return_loss=False)
    t = {"input": x, "text": cap["text"], "score": cap["score"], "seg_low": cap["seg_low"]}
    save_file({k: v.contiguous() for k, v in t.items()}, os.path.join(HERE, "tiny_ctx_eval.safetensors"))
    print("tiny_ctx: text norm", t["text"].norm().item())


def gen_full(name, b, h, w, keep_full_maps=(0, 11), cfg=CITYSCAPES_CFG, map_samples=256):
    model = build_reference(cfg).eval()
    cap = capture(model)
    x = images(b, h, w, seed=1234)
    with torch.no_grad():
        out = model(x, return_loss=False)
    t = {"input_stats": stats(x), "score": cap["score"], "text": cap["text"],
         "seg_low": cap["seg_low"], "depth_low": cap["depth_low"]}
    seg = out["seg"].flatten()
    idx = sample_idx(seg.numel(), 4096, seed=11)
    t["seg_idx"] = idx
    t["seg_val"] = seg[idx]
    t["seg_stats"] = stats(out["seg"])
    for i, mp in enumerate(cap["maps"]):
        t[f"map_stats{i}"] = stats(mp)
        fl = mp.flatten()
        ii = sample_idx(fl.numel(), map_samples, seed=100 + i)
        t[f"map_idx{i}"] = ii
        t[f"map_val{i}"] = fl[ii]
        if i in keep_full_maps:
            t[f"map{i}"] = mp
    save_file({k: v.contiguous() for k, v in t.items()}, os.path.join(HERE, f"{name}.safetensors"))
    print(name, "done")


def gen_vitl14():
    """BASELINE config 4 at a test size: 120x230 is not a multiple of the patch (14), so the
    patchify floor (8x16 grid, N = 129) is exercised too (models.py:543-556)."""
    gen_full("vitl14_1x120x230", 1, 120, 230, keep_full_maps=(0, 3), cfg=VITL14_CFG)


def gen_tokens():
    """Token ids of the 19 Cityscapes class names from the reference tokenizer
    (seg/denseclip/utils.py:301-314, context_length 6 as in the YAML)."""
    import json
    from denseclip.utils import tokenize
    t = tokenize(CITYSCAPES_CLASSES, context_length=6)
    toks = {c: [int(v) for v in t[i].tolist()] for i, c in enumerate(CITYSCAPES_CLASSES)}
    with open(os.path.join(HERE, "cityscapes_tokens.json"), "w") as f:
        json.dump({"context_length": 6, "tokens": toks, "sot": 49406, "eot": 49407}, f, indent=1)


def gen_manifest():
    """state_dict key -> (shape, dtype) of the reference model for both configs."""
    import json
    man = {}
    for name, cfg in (("tiny", TINY_CFG), ("tiny_ctx", TINY_CTX_CFG), ("cityscapes", CITYSCAPES_CFG),
                      ("vitl14", VITL14_CFG), ("mid", MID_CFG)):
        from denseclip import DenseCLIP
        sd = DenseCLIP(class_names=CITYSCAPES_CLASSES, **dict(cfg)).state_dict()
        man[name] = {k: [list(v.shape), str(v.dtype)] for k, v in sd.items()}
    with open(os.path.join(HERE, "state_dict_manifest.json"), "w") as f:
        json.dump(man, f, indent=0)


if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count())
    install_shims()
    if sys.argv[1:] == ["ctx"]:
        gen_manifest()
        gen_tiny_ctx()
        sys.exit(0)
    if sys.argv[1:] == ["cfg1"]:
        gen_full("vitb16_2x512x1024", 2, 512, 1024, keep_full_maps=(0, 11))
        sys.exit(0)
    if sys.argv[1:] == ["full8193"]:
        # BASELINE config 1's resolution (1024x2048 -> N = 8193 tokens, the CLS-split attention
        # kernels the benchmark runs) on one image: pre-upsample seg / depth, the score map, and
        # 2048 sampled elements + stats of each of the 12 read-out maps (full maps would be 25 MB each)
        gen_full("vitb16_1x1024x2048", 1, 1024, 2048, keep_full_maps=(), map_samples=2048)
        sys.exit(0)
    if sys.argv[1:] == ["vitl14"]:
        gen_manifest()
        gen_vitl14()
        sys.exit(0)
    if sys.argv[1:] == ["mid"]:
        gen_manifest()
        gen_mid()
        sys.exit(0)
    gen_tokens()
    gen_manifest()
    gen_tiny()
    gen_tiny_ctx()
    gen_mid()
    gen_full("vitb16_1x128x256", 1, 128, 256)
    gen_full("vitb16_2x512x1024", 2, 512, 1024, keep_full_maps=(0, 11))
    gen_vitl14()
