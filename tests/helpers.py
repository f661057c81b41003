"""Shared helpers for the test-suite: fixture loading, weight regeneration, metrics."""
import json
import os
import sys

import torch
from safetensors.torch import load_file

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
GOLDEN = os.path.join(TESTS, "golden")
for p in (ROOT, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)

from weights_spec import value_for  # noqa: E402
from model_configs import (TINY_CFG, TINY_CTX_CFG, CTX_GAMMA, CITYSCAPES_CFG, CITYSCAPES_CLASSES,  # noqa: E402,F401
                           VITL14_CFG, MID_CFG)


def manifest(name):
    with open(os.path.join(GOLDEN, "state_dict_manifest.json")) as f:
        return json.load(f)[name]


_DT = {"torch.float32": torch.float32, "torch.int64": torch.int64}


def spec_state_dict(name, seed=0):
    """Reference-keyed state dict filled from weights_spec (what the fixtures used)."""
    sd = {}
    for k, (shape, dt) in manifest(name).items():
        if dt == "torch.float32":
            sd[k] = value_for(k, shape, seed)
        else:
            sd[k] = torch.zeros(shape, dtype=_DT[dt])
    if name == "tiny_ctx":
        sd["gamma"] = torch.full_like(sd["gamma"], CTX_GAMMA)  # as gen_golden.gen_tiny_ctx
    return sd


def golden(name):
    return load_file(os.path.join(GOLDEN, name + ".safetensors"))


def class_tokens():
    with open(os.path.join(GOLDEN, "cityscapes_tokens.json")) as f:
        t = json.load(f)
    return torch.tensor([t["tokens"][c] for c in CITYSCAPES_CLASSES], dtype=torch.long)


def images(b, h, w, seed=1234):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(b, 3, h, w, generator=g)


def rel_err(a, b):
    """Norm-wise relative error ||a-b|| / ||b|| in fp64."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


def stats(t):
    t = t.double()
    return torch.tensor([t.mean(), t.std(), t.norm(), t.abs().max()], dtype=torch.float64)
