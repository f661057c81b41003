"""World-size-2 data-parallel step on CPU (gloo): the N > 1 path of bench.py / train.py.

The HIP ViT cannot run on a CPU host, so the DDP-wrapped module here is the trainable set
of the reference regime (mode R: neck + decode head + depth head, train_denseclip.py:
1040-1044) fed with per-rank feature maps; everything around it is the package's own
data-parallel code (train.wrap_ddp, train.loss_fn, train.make_optimizer, utils.
init_distributed).  Checked: rank-sharded batches average to the single-process gradient
of the concatenated batch (DDP all-reduce = weak scaling with fixed per-rank work), and the
AdamW step leaves both ranks with identical parameters.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from helpers import TINY_CFG, TINY_CTX_CFG, CITYSCAPES_CLASSES, rel_err


class _HeadsOnly(nn.Module):
    """neck -> decode/depth heads -> resize to the label size (DenseCLIP._heads + the
    train-branch resize of denseclip.py:838-868), on given maps."""

    def __init__(self, model):
        super().__init__()
        self.neck, self.decode_head, self.depth_head = model.neck, model.decode_head, model.depth_head

    def forward(self, maps, gt_semantic_seg=None, gt_depth=None, return_loss=True):
        x = self.neck(list(maps.unbind(0)))
        x = x[0] if isinstance(x, (list, tuple)) else x
        hw = gt_semantic_seg.shape[-2:]
        seg = F.interpolate(self.decode_head(x), size=hw, mode="bilinear", align_corners=False)
        depth = F.interpolate(self.depth_head(x), size=hw, mode="bilinear", align_corners=False)
        return {"main_output": seg, "depth_output": depth, "aux_losses": {}}


def _model():
    from denseclip_vit_multimodal_amd import DenseCLIP
    from denseclip_vit_multimodal_amd.train import freeze_for_mode
    torch.manual_seed(0)
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **TINY_CFG)
    trainable = freeze_for_mode(m, "R")
    names = {n for n, p in m.named_parameters() if p.requires_grad}
    # the reference rule (train_denseclip.py:1040-1044): everything but backbone.* / text_encoder.*
    assert names == {n for n, _ in m.named_parameters() if not n.startswith(("backbone.", "text_encoder."))}
    assert len(trainable) == len(names)
    h = _HeadsOnly(m)
    h.eval()  # BN batch statistics are per-rank in the reference too; eval keeps the check exact
    for mod in h.modules():
        for p in mod.parameters(recurse=False):
            p.requires_grad_(True)
    # a frozen parameter (like text_encoder.* / backbone.* in mode R): not reduced, but broadcast
    # from rank 0 at wrap time all the same (DDP's _sync_module_states)
    h.frozen = nn.Parameter(torch.linspace(-1, 1, 7), requires_grad=False)
    return h


def _batch(rank, B=2, layers=3, C=128, h=4, w=8, H=16, W=32):
    from denseclip_vit_multimodal_amd.train import synth_batch
    g = torch.Generator().manual_seed(100 + rank)
    maps = torch.randn(layers, B, C, h, w, generator=g)
    _, seg, depth, mask = synth_batch(B, H, W, torch.device("cpu"), rank=rank, image_dtype=torch.float32)
    return maps, seg, depth, mask


def _worker(rank, world, port, out_dir, impl=None, bucket_mb=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    from denseclip_vit_multimodal_amd.utils import init_distributed, cleanup
    from denseclip_vit_multimodal_amd.train import GradAllReduce, wrap_ddp, loss_fn, make_optimizer
    init_distributed(rank, world, backend="gloo")
    try:
        m = _model()
        with torch.no_grad():  # rank 1 starts elsewhere: wrapping broadcasts rank 0's parameters
            for p in m.parameters():
                p.add_(float(rank))
        from denseclip_vit_multimodal_amd import ops
        walks = []
        ops_set = ops.set_gemm_walk

        def record(w):
            walks.append(w)
            return ops_set(w)

        ops.set_gemm_walk = record
        model = GradAllReduce(m, bucket_cap_mb=bucket_mb) if bucket_mb else wrap_ddp(m, impl=impl)
        if bucket_mb:
            assert len(model._buckets) >= 5, len(model._buckets)
        opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
        with torch.no_grad():  # rank 1's BN statistics off: the wrapper's forward restores rank 0's
            for b in model.module.buffers():
                if b.is_floating_point():
                    b.add_(float(rank))
        maps, seg, depth, mask = _batch(rank)
        out = model(maps, gt_semantic_seg=seg, gt_depth=depth)
        loss = loss_fn(out, seg, depth, mask)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        ops.set_gemm_walk = ops_set
        grads = {n: p.grad.clone() for n, p in model.module.named_parameters() if p.requires_grad}
        opt.step()
        params = {n: p.detach().clone() for n, p in model.module.named_parameters()}
        bufs = {n: b.clone() for n, b in model.module.named_buffers()}
        torch.save({"grads": grads, "params": params, "loss": loss.detach(), "buffers": bufs,
                    "walks": torch.tensor(walks, dtype=torch.int64)},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        cleanup()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("impl,bucket_mb", [("allreduce", None), ("ddp", None), ("allreduce", 0.01)],
                         ids=["allreduce", "ddp", "allreduce_many_buckets"])
def test_ddp_world2_matches_single_process(tmp_path, impl, bucket_mb):
    """Both data-parallel implementations of wrap_ddp (train.GradAllReduce, the default, and torch
    DDP), and GradAllReduce with ~10 KB buckets (six buckets, each launched as its last
    gradient lands): averaged gradients = the single-process gradient of the concatenated batch,
    identical parameters on both ranks after the step, rank 0's parameters broadcast at wrap time
    and its buffers before the forward (rank 1 starts with different values of both)."""
    from denseclip_vit_multimodal_amd.train import loss_fn
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), impl, bucket_mb), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"rank{i}.pt", weights_only=True) for i in range(world)]

    # single process: mean of the per-rank losses over the same shards (same thread count
    # as the workers, so oneDNN picks the same conv algorithms)
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    ref = _model()
    total = 0
    for rank in range(world):
        maps, seg, depth, mask = _batch(rank)
        out = ref(maps, gt_semantic_seg=seg, gt_depth=depth)
        total = total + loss_fn(out, seg, depth, mask)
    (total / world).backward()
    torch.set_num_threads(nt)
    for n, p in ref.named_parameters():
        if not p.requires_grad:
            continue
        for i in range(world):
            g = r[i]["grads"][n]
            assert rel_err(g, p.grad) < 1e-4, (n, i, rel_err(g, p.grad))  # fp32 sum-order noise only
    for n in r[0]["params"]:
        assert torch.equal(r[0]["params"][n], r[1]["params"][n]), n
    # the frozen parameter: rank 1's perturbed copy was replaced by rank 0's at wrap time
    assert torch.equal(r[1]["params"]["frozen"], torch.linspace(-1, 1, 7))
    if impl == "allreduce":
        # the GEMM tile walk: claims (1) from the first bucket's collective to the end of the
        # backward, then back to the static walk (0)
        for i in range(world):
            assert r[i]["walks"].tolist() == [1, 0], r[i]["walks"]
    assert not torch.equal(r[0]["loss"], r[1]["loss"])  # the shards really differ
    rb = dict(ref.named_buffers())
    assert rb and set(rb) == set(r[1]["buffers"])
    for n, b in rb.items():  # rank 1's perturbed buffers were overwritten with rank 0's
        assert torch.equal(r[1]["buffers"][n], b) and torch.equal(r[0]["buffers"][n], b), n


def test_rank_shards_are_distinct():
    from denseclip_vit_multimodal_amd.train import synth_batch
    a = synth_batch(1, 32, 64, torch.device("cpu"), rank=0, image_dtype=torch.float32)
    b = synth_batch(1, 32, 64, torch.device("cpu"), rank=1, image_dtype=torch.float32)
    a2 = synth_batch(1, 32, 64, torch.device("cpu"), rank=0, image_dtype=torch.float32)
    assert all(torch.equal(x, y) for x, y in zip(a, a2))
    assert not torch.equal(a[0], b[0]) and not torch.equal(a[1], b[1])
    seg = a[1]
    frac_ignore = float((seg == 255).float().mean())
    assert 0.05 < frac_ignore < 0.15 and int(seg[seg != 255].max()) < 19


@pytest.mark.parametrize("cfg", [TINY_CFG, TINY_CTX_CFG, dict(TINY_CTX_CFG, score_concat_index=2)],
                         ids=["tiny", "ctx", "ctx_concat2"])
def test_wrap_ddp_leaves_gradless_parameters_out(tmp_path, cfg):
    """wrap_ddp on the whole DenseCLIP (gloo, world size 1): the trainable parameters that get no
    gradient (the no_grad score branch — contexts, gamma, projections, ContextDecoder — for any
    score_concat_index, and the unused CLIP projection; top-level ones included — DDP names them
    '.gamma') are not in the reducer, everything else trainable is.  The two-step DDP run of such a
    config is tests/test_gpu_dropin_heads.py::test_score_concat_and_context_decoder_train_under_ddp."""
    import torch.distributed as dist
    from denseclip_vit_multimodal_amd import DenseCLIP
    from denseclip_vit_multimodal_amd.train import freeze_for_mode, gradless_parameter_names, wrap_ddp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **cfg)
        freeze_for_mode(m, "F")
        dead = set(gradless_parameter_names(m))
        assert {"gamma", "contexts", "backbone.proj"} <= dead
        cd = {n for n, _ in m.named_parameters() if n.startswith("context_decoder.")}
        assert cd <= dead and (cd or cfg.get("context_decoder") is None)
        ddp = wrap_ddp(m)
        managed = {id(p) for p in ddp._module_parameters}
        for n, p in m.named_parameters():
            assert (id(p) in managed) == (n not in dead), n
    finally:
        dist.destroy_process_group()


def _skip_worker(rank, world, port, out_dir, fused):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    from denseclip_vit_multimodal_amd.utils import init_distributed, cleanup
    from denseclip_vit_multimodal_amd.train import step_unless_nonfinite
    init_distributed(rank, world, backend="gloo")
    try:
        w = torch.nn.Parameter(torch.ones(5))
        opt = torch.optim.AdamW([w], lr=0.1, fused=fused)
        w.grad = torch.full((5,), 0.5)  # all-reduced gradients are identical on every rank
        loss = torch.tensor(float("nan") if rank == 1 else 1.0)  # only rank 1's local loss is NaN
        step_unless_nonfinite(opt, loss)
        torch.save({"w": w.detach().clone()}, os.path.join(out_dir, f"skip{rank}.pt"))
    finally:
        cleanup()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fused", [False, True], ids=["foreach", "fused"])
def test_nonfinite_skip_is_rank_consistent(tmp_path, fused):
    """one rank's non-finite loss skips the step on EVERY rank (the flag is MAX-reduced
    for non-fused optimizers too), so the replicas stay identical."""
    world = 2
    mp.spawn(_skip_worker, args=(world, _free_port(), str(tmp_path), fused), nprocs=world, join=True)
    for i in range(world):
        w = torch.load(tmp_path / f"skip{i}.pt", weights_only=True)["w"]
        assert torch.equal(w, torch.ones(5)), (i, w)


def test_grad_allreduce_issues_buckets_in_bucket_order():
    """collectives are issued in bucket order whatever order autograd
    completes the buckets in (a bucket that completes early waits for its predecessors), so
    every rank issues the same sequence; a bucket with a parameter that got no gradient is
    issued by _finish, still in order."""
    import torch.distributed as dist
    from denseclip_vit_multimodal_amd.train import GradAllReduce
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        m = nn.Sequential(*[nn.Linear(64, 64) for _ in range(6)])
        w = GradAllReduce(m, bucket_cap_mb=0.01, last_bucket_cap_mb=0.01)
        nb = len(w._buckets)
        assert nb >= 4
        order = []
        w._launch = lambda i: (order.append(i), w._pending["launched"].__setitem__(i, True))
        # the state _on_grad creates at the first gradient of a backward (outside a backward
        # there is no engine to queue _finish on, so seed it here)
        w._pending = {"ready": [0] * nb, "launched": [False] * nb, "works": [], "next": 0, "walk": None}
        # complete bucket 2 first, then 0, then every bucket but the last's last parameter
        feed = list(w._buckets[2]) + list(w._buckets[0]) + [p for i in range(nb) if i not in (0, 2)
                                                             for p in w._buckets[i]][:-1]
        with torch.no_grad():
            for p in feed:
                w._on_grad(p)
        assert order == list(range(nb - 1)), order
        w._finish()
        assert order == list(range(nb)), order
    finally:
        dist.destroy_process_group()
