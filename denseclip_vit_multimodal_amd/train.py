"""Data-parallel train step of the reference trainer, restated for one process per GPU.

What `seg/train_denseclip.py` does around the hot path, kept to the parts that shape the
step (its CLI, logging, metrics and checkpointing are out of scope — DESIGN.md §7):
  * freeze rule            train_denseclip.py:1040-1044 (backbone.* and text_encoder.*)
  * DDP wrap               train_denseclip.py:1050-1054 (gradient all-reduce over RCCL)
  * loss                   train_denseclip.py:1086-1095, 1265-1314: CE(ignore 255) + 0.1 SILog
  * optimiser              train_denseclip.py:1061: AdamW(lr 2e-5, weight decay 0.01)
  * per-rank data          DistributedSampler (train_denseclip.py:242): rank r sees its own
                           shard; here synthetic Cityscapes-shaped tensors seeded per rank
                           (real data: data.CityscapesDepthSegDataset + data.prepare_batch).
  * checkpoints            train_denseclip.py:1012-1034 (--load), 1107-1133 (--resume),
                           1491-1521 (save): {'epoch', 'state_dict', 'optimizer'[, 'scheduler']}.
Mode "R" is the reference regime (backbone + text frozen); mode "F" also trains the ViT,
which exercises the HIP backward kernels (the north star's roofline applies there).
"""
import torch
import torch.nn.functional as F

from .losses import SILogLoss

# parameters that feed nothing differentiable in the ViT Cityscapes config: the unused
# CLIP projection and the score-map branch, whose output is discarded (denseclip.py:747)
_DEAD = ("backbone.proj", "contexts", "gamma")
_DEAD_PREFIX = ("vis_proj.", "global_proj.")


def freeze_for_mode(model, mode):
    """requires_grad per the reference freeze rule; returns the trainable parameters."""
    if mode not in ("F", "R"):
        raise ValueError(f"mode must be 'F' or 'R' (got {mode!r})")
    params = []
    for name, p in model.named_parameters():
        frozen = name.startswith("text_encoder.")
        if mode == "R":
            frozen = frozen or name.startswith("backbone.")
        if name in _DEAD or name.startswith(_DEAD_PREFIX):
            frozen = True
        p.requires_grad_(not frozen)
        if not frozen:
            params.append(p)
    return params


def synth_batch(B, H, W, device, rank=0, image_dtype=torch.bfloat16, num_classes=19):
    """Rank-seeded synthetic Cityscapes-shaped batch (images randn seed 1234,
    seg labels with 10 % ignore (255) seed 1235, depth U(1, 80) with 20 % invalid seed 1236)."""
    g = torch.Generator(device="cpu").manual_seed(1234 + rank)
    img = torch.randn(B, 3, H, W, generator=g).to(device).to(image_dtype)
    g = torch.Generator(device="cpu").manual_seed(1235 + rank)
    seg = torch.randint(0, num_classes, (B, H, W), generator=g)
    seg[torch.rand(B, H, W, generator=g) < 0.1] = 255
    g = torch.Generator(device="cpu").manual_seed(1236 + rank)
    depth = 1 + 79 * torch.rand(B, 1, H, W, generator=g)
    mask = torch.rand(B, 1, H, W, generator=g) >= 0.2
    return img, seg.to(device), depth.to(device), mask.to(device)


def loss_fn(out, seg, depth, mask, silog=None):
    """CE(ignore 255) + 0.1 * SILog (train_denseclip.py:1265-1314).  With a model in
    fused_head_loss mode the outputs are the heads' low-res maps and the resize + loss run
    as one fused kernel each (identical loss and gradients)."""
    silog = silog or SILogLoss()
    if out.get("main_output_lowres") is not None:
        from . import ops
        loss = ops.UpsampleCEFn.apply(out["main_output_lowres"], seg, 255)
        if out.get("depth_output_lowres") is not None:
            loss = loss + 0.1 * ops.UpsampleSILogFn.apply(out["depth_output_lowres"], depth, mask, silog.lambd,
                                                          silog.eps)
        return loss
    loss = F.cross_entropy(out["main_output"], seg, ignore_index=255)
    if out.get("depth_output") is not None:
        loss = loss + 0.1 * silog(out["depth_output"], depth, mask)
    return loss


def wrap_ddp(model, device=None):
    """DDP over the default process group (RCCL on GPUs, gloo on CPU).  100 MB buckets:
    fewer, larger all-reduces suit xGMI's per-link ring bandwidth; the buckets are views of
    the gradients (no copy)."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    ids = [device.index] if device is not None and device.type == "cuda" else None
    return DDP(model, device_ids=ids, bucket_cap_mb=100, gradient_as_bucket_view=True,
               find_unused_parameters=False)


def make_optimizer(params, fused=None):
    if fused is None:
        fused = all(p.is_cuda for p in params)
    return torch.optim.AdamW(params, lr=2e-5, weight_decay=0.01, fused=fused)


def train_step(model, opt, batch, silog=None):
    """One step: forward (DenseCLIP.forward train branch), loss, backward (DDP all-reduce
    overlapped with it), AdamW.  Returns the loss tensor (no host sync)."""
    img, seg, depth, mask = batch
    out = model(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True)
    loss = loss_fn(out, seg, depth, mask, silog)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
    return loss.detach()


# ---------------------------------------------------------------------------- checkpoints
def _unwrap(model):
    return model.module if hasattr(model, "module") else model


def save_checkpoint(path, model, optimizer, epoch, scheduler=None):
    """The reference trainer's checkpoint (train_denseclip.py:1499-1512): the UNWRAPPED model's
    state dict (no 'module.' prefix), the optimizer's and optionally the scheduler's."""
    state = {"epoch": epoch, "state_dict": _unwrap(model).state_dict(), "optimizer": optimizer.state_dict()}
    if scheduler is not None:
        state["scheduler"] = scheduler.state_dict()
    torch.save(state, path)


def _model_weights(ckpt):
    """Weight dict of a checkpoint as --load reads it (train_denseclip.py:1019-1021): under
    'state_dict', 'model_state_dict' or 'model', or the dict itself; a 'module.' prefix on every
    key (a DDP-saved model) is stripped."""
    for key in ("state_dict", "model_state_dict", "model"):
        if key in ckpt:
            ckpt = ckpt[key]
            break
    if ckpt and all(k.startswith("module.") for k in ckpt):
        ckpt = {k[len("module."):]: v for k, v in ckpt.items()}
    return ckpt


def load_weights(path, model, map_location="cpu"):
    """--load (train_denseclip.py:1012-1024): non-strict load of a checkpoint's model weights;
    returns the load message.  Files are read with weights_only=True; an unreadable file raises
    (the reference logs and continues)."""
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    return _unwrap(model).load_state_dict(_model_weights(ckpt), strict=False)


def resume(path, model, optimizer=None, scheduler=None, map_location="cpu"):
    """--resume (train_denseclip.py:1107-1133): model, optimizer and scheduler state; returns the
    epoch to start from (saved epoch + 1)."""
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    if "state_dict" in ckpt:
        _unwrap(model).load_state_dict(_model_weights(ckpt), strict=False)
    if optimizer is not None and "optimizer" in ckpt:
        optimizer.load_state_dict(ckpt["optimizer"])
    if scheduler is not None and "scheduler" in ckpt:
        scheduler.load_state_dict(ckpt["scheduler"])
    return ckpt.get("epoch", -1) + 1
