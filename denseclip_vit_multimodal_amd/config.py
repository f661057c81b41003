"""YAML config loading with the reference trainer's semantics (train_denseclip.py:958-1005):
the `model` section minus `type`/`pretrained`/`init_cfg`/... becomes DenseCLIP(**kwargs)
with `clip_pretrained` -> clip_pretrained_path and `context_length`, `text_dim`,
`token_embed_dim` passed explicitly."""
import os

import yaml

_HERE = os.path.dirname(os.path.abspath(__file__))
CONFIG_DIR = os.path.join(_HERE, "configs")

CITYSCAPES_CLASSES = [
    'road', 'sidewalk', 'building', 'wall', 'fence', 'pole',
    'traffic light', 'traffic sign', 'vegetation', 'terrain', 'sky',
    'person', 'rider', 'car', 'truck', 'bus', 'train',
    'motorcycle', 'bicycle',
]


def load_yaml(path):
    if not os.path.exists(path) and os.path.exists(os.path.join(CONFIG_DIR, path)):
        path = os.path.join(CONFIG_DIR, path)
    with open(path) as f:
        return yaml.safe_load(f)


def model_kwargs(cfg, clip_path_override=None):
    """The kwargs train_denseclip.py passes to DenseCLIP (without class_names)."""
    m = dict(cfg["model"])
    if m.get("type", "DenseCLIP") != "DenseCLIP":
        raise ValueError(f"Model type '{m.get('type')}' not recognized.")
    for k in ("pretrained", "init_cfg", "train_cfg", "test_cfg", "download_dir", "type"):
        m.pop(k, None)
    out = {}
    for k in ("backbone", "text_encoder", "decode_head", "context_decoder", "neck", "auxiliary_head",
              "identity_head", "depth_head"):
        out[k] = m.pop(k, None)
    clip = m.pop("clip_pretrained", None)
    out["clip_pretrained_path"] = clip_path_override if clip_path_override is not None else clip
    ctx_len = m.pop("context_length", None)
    out["context_length"] = ctx_len if ctx_len is not None else cfg["model"].get("context_length", 77)
    m.pop("text_dim", None)
    m.pop("token_embed_dim", None)
    out["token_embed_dim"] = cfg["model"].get("token_embed_dim", 512)
    out["text_dim"] = cfg["model"].get("text_dim", 512)
    out.update(m)
    return out


def build_model(cfg, class_names=None, clip_path_override=None):
    from .denseclip import DenseCLIP
    kw = model_kwargs(cfg, clip_path_override)
    if kw["clip_pretrained_path"] and not os.path.exists(kw["clip_pretrained_path"]):
        kw["clip_pretrained_path"] = None  # the reference logs and continues (denseclip.py:190)
    return DenseCLIP(class_names=class_names or CITYSCAPES_CLASSES, **kw)
