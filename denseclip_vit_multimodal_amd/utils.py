"""Training utilities and the CLIP tokenizer (reference seg/denseclip/utils.py).

`init_distributed` is the data-parallel comm backend: one process per GPU, backend
"nccl" (= RCCL on ROCm) over xGMI.  Unlike the reference (utils.py:102-107, hard-coded
localhost:12355) it honours MASTER_ADDR/MASTER_PORT from torchrun when present.
"""
import gzip
import html
import json
import logging
import os
import platform
import random
from functools import lru_cache

import numpy as np
import torch
import torch.distributed as dist

try:
    import regex as re
except ImportError:  # pragma: no cover
    import re

_HERE = os.path.dirname(os.path.abspath(__file__))


def setup_logger(log_dir, rank=0):
    """Rank-aware file + console logger (reference utils.py:30-49)."""
    os.makedirs(log_dir, exist_ok=True)
    logger = logging.getLogger("DenseCLIP")
    logger.setLevel(logging.INFO if rank == 0 else logging.WARN)
    fmt = logging.Formatter("%(asctime)s - %(levelname)s - %(message)s")
    fh = logging.FileHandler(os.path.join(log_dir, f"training_rank{rank}.log"))
    fh.setFormatter(fmt)
    logger.addHandler(fh)
    if rank == 0:
        ch = logging.StreamHandler()
        ch.setFormatter(fmt)
        logger.addHandler(ch)
    return logger


def set_random_seed(seed, deterministic=False):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    if deterministic:
        torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False


def init_distributed(rank, world_size, backend=None):
    """One process per GPU; RCCL ('nccl') on GPUs, gloo on CPU-only hosts."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "12355")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(rank % torch.cuda.device_count())
    dist.init_process_group(backend, rank=rank, world_size=world_size)


def cleanup():
    if dist.is_initialized():
        dist.destroy_process_group()


def collect_env_info():
    lines = [f"PyTorch: {torch.__version__}", f"HIP: {getattr(torch.version, 'hip', None)}",
             f"GPU available: {torch.cuda.is_available()}", f"OS: {platform.system()} {platform.release()}"]
    if torch.cuda.is_available():
        lines.append(f"Device: {torch.cuda.get_device_name(0)} x{torch.cuda.device_count()}")
    return "\n".join(lines)


# ============================================================================ tokenizer
@lru_cache()
def bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


class SimpleTokenizer:
    """CLIP byte-level BPE (the published OpenAI CLIP algorithm, as used by reference
    utils.py:187-299).  Needs the 16e6 merges file (not shipped: pass `bpe_path` or set
    DENSECLIP_BPE_PATH)."""

    def __init__(self, bpe_path):
        self.byte_encoder = bytes_to_unicode()
        merges = gzip.open(bpe_path).read().decode("utf-8").split("\n")[1:49152 - 256 - 2 + 1]
        merges = [tuple(m.split()) for m in merges]
        vocab = list(self.byte_encoder.values())
        vocab = vocab + [v + "</w>" for v in vocab] + ["".join(m) for m in merges]
        vocab += ["<|startoftext|>", "<|endoftext|>"]
        self.encoder = {v: i for i, v in enumerate(vocab)}
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.cache = {}
        self.pat = re.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""",
                              re.IGNORECASE)

    def bpe(self, token):
        if token in self.cache:
            return self.cache[token]
        word = list(token[:-1]) + [token[-1] + "</w>"]
        while len(word) > 1:
            pairs = {(word[i], word[i + 1]) for i in range(len(word) - 1)}
            best = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if best not in self.bpe_ranks:
                break
            merged, i = [], 0
            while i < len(word):
                if i < len(word) - 1 and (word[i], word[i + 1]) == best:
                    merged.append(word[i] + word[i + 1])
                    i += 2
                else:
                    merged.append(word[i])
                    i += 1
            word = merged
        self.cache[token] = word
        return word

    def encode(self, text):
        text = re.sub(r"\s+", " ", html.unescape(html.unescape(text)).strip()).strip().lower()
        out = []
        for tok in re.findall(self.pat, text):
            tok = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            out.extend(self.encoder[t] for t in self.bpe(tok))
        return out


SOT, EOT = 49406, 49407


@lru_cache()
def _known_tokens():
    with open(os.path.join(_HERE, "data", "clip_class_tokens.json")) as f:
        return json.load(f)["tokens"]


@lru_cache()
def _tokenizer():
    path = os.environ.get("DENSECLIP_BPE_PATH")
    if path and os.path.exists(path):
        return SimpleTokenizer(path)
    return None


def _encode(text):
    tk = _tokenizer()
    if tk is not None:
        return [SOT] + tk.encode(text) + [EOT]
    known = _known_tokens()
    if text in known:
        return [t for t in known[text] if t != 0]
    raise RuntimeError(f"no BPE vocabulary available to tokenize {text!r}: set DENSECLIP_BPE_PATH to CLIP's "
                       "bpe_simple_vocab_16e6.txt.gz (built-in table covers the Cityscapes class names)")


def tokenize(texts, context_length=77, truncate=False):
    """reference utils.py:301-314: SOT + BPE + EOT, zero padded to context_length."""
    if isinstance(texts, str):
        texts = [texts]
    result = torch.zeros(len(texts), context_length, dtype=torch.long)
    for i, t in enumerate(texts):
        toks = _encode(t)
        if len(toks) > context_length:
            if not truncate:
                raise RuntimeError(f"Input {t} is too long for context length {context_length}")
            toks = toks[:context_length]
            toks[-1] = EOT
        result[i, : len(toks)] = torch.tensor(toks)
    return result
