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

# parameters that never receive a gradient: the unused CLIP projection and everything the
# score-map branch touches — the learnable text contexts, gamma, vis_proj / global_proj and the
# ContextDecoder.  That branch runs under no_grad and its output is discarded for every
# score_concat_index (the reference concatenates the score map onto a clone of the maps that the
# forward never passes on, denseclip.py:586, 684-694, 747).  They stay trainable — the
# reference's AdamW param list holds them (train_denseclip.py:1040-1044, 1061), so optimizer
# states interoperate — and are kept out of the DDP gradient reduction instead.
_DEAD = ("backbone.proj", "contexts", "gamma")
_DEAD_PREFIX = ("vis_proj.", "global_proj.", "context_decoder.")


def gradless_parameter_names(model):
    """Trainable parameter names that get no gradient (DDP must not wait for them)."""
    return [n for n, p in _unwrap(model).named_parameters()
            if p.requires_grad and (n in _DEAD or n.startswith(_DEAD_PREFIX))]


def freeze_for_mode(model, mode):
    """requires_grad per the reference freeze rule (train_denseclip.py:1040-1044: backbone.* and
    text_encoder.* frozen; mode F also trains the backbone); returns the trainable parameters
    in named_parameters order — the reference optimizer's param list."""
    if mode not in ("F", "R"):
        raise ValueError(f"mode must be 'F' or 'R' (got {mode!r})")
    params = []
    for name, p in model.named_parameters():
        frozen = name.startswith("text_encoder.")
        if mode == "R":
            frozen = frozen or name.startswith("backbone.")
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


def loss_config(cfg):
    """(seg weight, silog weight, SILogLoss) from a trainer YAML (train_denseclip.py:1088-1095,
    1311-1312: training.loss_weights.{seg, silog}, training.silog_loss.{lambda, eps})."""
    tr = (cfg or {}).get("training", {}) or {}
    # the reference's defaults: the whole dict {'seg': 1.0, 'silog': 0.1} when absent, 1.0 for a
    # key missing from a given dict (train_denseclip.py:1094-1095, 1311-1312)
    w = tr.get("loss_weights", {"seg": 1.0, "silog": 0.1}) or {}
    sl = tr.get("silog_loss", {}) or {}
    return (float(w.get("seg", 1.0)), float(w.get("silog", 1.0)),
            SILogLoss(lambd=float(sl.get("lambda", 0.5)), eps=float(sl.get("eps", 1e-6))))


def loss_fn(out, seg, depth, mask, silog=None, seg_weight=1.0, silog_weight=0.1):
    """seg_weight * CE(ignore 255) + silog_weight * SILog (train_denseclip.py:1265-1314; the
    weights and the SILog parameters come from the config, `loss_config`).  With a model in
    fused_head_loss mode the outputs are the heads' low-res maps and the resize + loss run
    as one fused kernel each (identical loss and gradients).  A batch whose labels are all
    ignored gives a NaN CE, as torch's CrossEntropyLoss does (the reference trainer then
    skips the step, train_denseclip.py:1323)."""
    silog = silog or SILogLoss()
    if out.get("main_output_lowres") is not None:
        from . import ops
        loss = seg_weight * ops.UpsampleCEFn.apply(out["main_output_lowres"], seg, 255)
        if out.get("depth_output_lowres") is not None:
            loss = loss + silog_weight * ops.UpsampleSILogFn.apply(out["depth_output_lowres"], depth, mask,
                                                                   silog.lambd, silog.eps)
        return loss
    loss = seg_weight * F.cross_entropy(out["main_output"], seg, ignore_index=255)
    if out.get("depth_output") is not None:
        loss = loss + silog_weight * silog(out["depth_output"], depth, mask)
    return loss


# wrap_ddp's data-parallel implementation: "allreduce" (GradAllReduce: bucketed in-place
# all-reduces of the gradients autograd produced) or "ddp" (torch's DistributedDataParallel)
DP_IMPL = "allreduce"


def wrap_ddp(model, device=None, grad_dtype=None, impl=None):
    """Data parallelism over the default process group (RCCL on GPUs, gloo on CPU): GradAllReduce
    (DP_IMPL "allreduce", the default) or torch DDP ("ddp", and always for grad_dtype bf16).
    DDP: 100 MB buckets:
    fewer, larger all-reduces suit xGMI's per-link ring bandwidth; the buckets are views of
    the gradients (no copy).  Trainable parameters that get no gradient in this config
    (`gradless_parameter_names`) are left out of the reduction rather than searched for every
    step (find_unused_parameters).  grad_dtype=torch.bfloat16 all-reduces the buckets in bf16
    (half the xGMI bytes; the sum is rounded to 8 mantissa bits) via DDP's compression hook."""
    impl = impl or DP_IMPL
    if impl not in ("allreduce", "ddp"):
        raise ValueError(f"unknown data-parallel implementation {impl!r}")
    if impl == "allreduce" and grad_dtype in (None, torch.float32):
        return GradAllReduce(model)
    from torch.nn.parallel import DistributedDataParallel as DDP
    ignore = set(gradless_parameter_names(model))
    if ignore:
        # DDP matches both the named_parameters() name ("gamma") and f"{module_name}.{param_name}"
        # (".gamma" for a top-level parameter) in different places: give both forms
        fq = [f"{mn}.{pn}" for mn, mod in model.named_modules() for pn, _ in mod.named_parameters(recurse=False)
              if (f"{mn}.{pn}" if mn else pn) in ignore]
        DDP._set_params_and_buffers_to_ignore_for_model(model, sorted(ignore | set(fq)))
    ids = [device.index] if device is not None and device.type == "cuda" else None
    ddp = DDP(model, device_ids=ids, bucket_cap_mb=100, gradient_as_bucket_view=True,
              find_unused_parameters=False)
    if grad_dtype == torch.bfloat16:
        from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
        ddp.register_comm_hook(None, default_hooks.bf16_compress_hook)
    elif grad_dtype not in (None, torch.float32):
        raise ValueError(f"unsupported gradient all-reduce dtype {grad_dtype}")
    return ddp


class GradAllReduce(torch.nn.Module):
    """Data parallelism over the default process group without DDP's gradient copies: the same
    contract as wrap_ddp (parameters broadcast from rank 0 at wrap time, buffers before every
    forward, gradients averaged over the ranks before the optimizer step, overlapped with the
    backward, ~100 MB buckets in reverse registration order — the last to complete ~25 MB, so
    little is left exposed after the backward — the gradless parameters left out)
    — but each bucket's collective runs on the gradient tensors autograd produced, in place.

    Why: DDP keeps a flat bucket per ~100 MB and copies every gradient into it (or accumulates
    into bucket views): at ViT-B/16 ~250 device copies and ~100 fills per step, +3 % of the step at
    world size 1 (profiles/r05/r5ac) — a fixed cost of every N > 1 step.  Here a post-accumulate-
    grad hook counts each bucket's arrivals; the bucket whose last gradient lands is reduced at
    once (RCCL: one coalesced group of in-place AVG all-reduces on the process group's stream; gloo:
    SUM then / world), and a callback queued on the autograd engine waits for every bucket at the
    end of the backward (the current stream waits on the collectives' stream; no host sync for
    RCCL).  Gradients of `set_to_none` steps are stolen by autograd, so nothing is copied."""

    def __init__(self, module, bucket_cap_mb=100, broadcast_buffers=True, last_bucket_cap_mb=25):
        super().__init__()
        import torch.distributed as dist
        self.module = module
        self._dist = dist
        ignore = set(gradless_parameter_names(module))
        params = [(n, p) for n, p in module.named_parameters() if p.requires_grad and n not in ignore]
        # the parameters not ignored (DDP's attribute: frozen ones included; only those with
        # requires_grad are reduced)
        self._module_parameters = [p for n, p in module.named_parameters() if n not in ignore]
        from torch.distributed.distributed_c10d import _get_default_group
        if self._module_parameters and dist.get_world_size() > 1:
            # rank 0's initial parameters, flattened into ~250 MB broadcasts: EVERY parameter not
            # ignored, frozen ones included, as DDP's _sync_module_states does (the reference seeds
            # each rank with seed + rank, train_denseclip.py:941, so a randomly initialised frozen
            # weight would otherwise differ between ranks)
            with torch.no_grad():
                dist._broadcast_coalesced(_get_default_group(), [p.data for p in self._module_parameters],
                                          250 * 2 ** 20, 0)
        self._buffers_to_sync = [b for b in module.buffers()] if broadcast_buffers else []
        # gradients arrive roughly in reverse registration order, so the bucket of the FIRST
        # registered parameters (patch embedding, block 0) completes last and its all-reduce is the
        # one left exposed after the backward: it is cut at last_bucket_cap_mb (~block 0 at
        # ViT-B/16), the others at bucket_cap_mb (few, large collectives for xGMI's ring links)
        caps = (min(last_bucket_cap_mb, bucket_cap_mb) * 2 ** 20, bucket_cap_mb * 2 ** 20)
        fwd, cur, size = [], [], 0
        for _, p in params:
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= caps[1 if fwd else 0]:
                fwd.append(cur)
                cur, size = [], 0
        if cur:
            fwd.append(cur)
        self._buckets = [list(reversed(b)) for b in reversed(fwd)]  # in the order they complete
        self._bucket_of = {}
        for i, b in enumerate(self._buckets):
            for p in b:
                self._bucket_of[p] = i
        self._nccl = dist.get_backend() == "nccl"
        self._world = dist.get_world_size()
        # one rank: the average is the identity and no collective is issued (set False to exercise
        # the collective path anyway — bench.py's ddp1 line prices RCCL's one-rank all-reduce so)
        self.skip_collectives = self._world == 1
        self.coalesce = True  # RCCL: a bucket's all-reduces as one group call
        # the persistent GEMMs' tile walk while a bucket's collective is in flight (DCLIP_OPT_GEMM_SCHED
        # value: 1 = every tile claimed, so the workgroups that find a CU held by RCCL's channel
        # kernels leave their tiles to the others; None keeps whatever walk is set).  The static walk
        # is faster uncontended (+4 % for claims) but loses 49 % vs 22 % with 16 CUs held
        # (profiles/r05/r5e_ab_gemm_walks.log), and the buckets complete through the whole backward,
        # so the GEMMs launched between the first bucket's launch and _finish take the claims walk
        self.gemm_walk_under_collectives = 1
        self._pending = None
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for _, p in params]

    def forward(self, *args, **kwargs):
        if self._buffers_to_sync and self._world > 1:
            # rank 0's buffers (BN running statistics: 45 small tensors at ViT-B/16) in one
            # flattened broadcast per dtype, as DDP's buffer sync does — not one collective each
            from torch.distributed.distributed_c10d import _get_default_group
            with torch.no_grad():
                self._dist._broadcast_coalesced(_get_default_group(), self._buffers_to_sync, 250 * 2 ** 20, 0)
        self._pending = None
        return self.module(*args, **kwargs)

    def _launch(self, i):
        grads = [p.grad for p in self._buckets[i] if p.grad is not None]
        st = self._pending
        st["launched"][i] = True
        if not grads or self.skip_collectives:
            return
        if st["walk"] is None and self.gemm_walk_under_collectives is not None:
            from . import ops
            st["walk"] = ops.set_gemm_walk(self.gemm_walk_under_collectives)
        d = self._dist
        if self._nccl and self.coalesce:
            with d._coalescing_manager(async_ops=True) as cm:
                for g in grads:
                    d.all_reduce(g, op=d.ReduceOp.AVG)
            st["works"].append((cm, None))
        elif self._nccl:  # one async call per tensor
            for g in grads:
                st["works"].append((d.all_reduce(g, op=d.ReduceOp.AVG, async_op=True), None))
        else:
            for g in grads:
                st["works"].append((d.all_reduce(g, async_op=True), g))

    def _on_grad(self, p):
        if self._pending is None:
            self._pending = {"ready": [0] * len(self._buckets), "launched": [False] * len(self._buckets), "works": [],
                             "next": 0, "walk": None}
            torch.autograd.Variable._execution_engine.queue_callback(self._finish)
        i = self._bucket_of[p]
        st = self._pending
        st["ready"][i] += 1
        # collectives are issued in BUCKET order, as DDP's reducer does: a bucket that completes
        # early waits for its predecessors, so every rank issues the same sequence of collectives
        # even if autograd visits the parameters in a different order on some rank
        while st["next"] < len(self._buckets) and st["ready"][st["next"]] == len(self._buckets[st["next"]]):
            self._launch(st["next"])
            st["next"] += 1

    def _finish(self):
        st = self._pending
        if st is None:
            return
        for i, done in enumerate(st["launched"]):
            if not done:  # a bucket some of whose parameters got no gradient this step (bucket order)
                self._launch(i)
        for w, g in st["works"]:
            w.wait()
            if g is not None:  # gloo has no AVG
                g.div_(self._world)
        if st["walk"] is not None:  # the current stream now waits on the collectives: back to the walk before
            from . import ops
            ops.set_gemm_walk(st["walk"])
        self._pending = None


def make_optimizer(params, fused=None, capturable=False):
    """AdamW(lr 2e-5, weight decay 0.01) as the reference trainer builds it (train_denseclip.py:1061),
    fused on GPU parameters; capturable=True keeps its step counts on the device (required by
    CapturedTrainStep)."""
    params = list(params)
    if fused is None:
        fused = all(p.is_cuda for p in params)
    if capturable:
        return torch.optim.AdamW(params, lr=2e-5, weight_decay=0.01, fused=fused, capturable=True)
    return torch.optim.AdamW(params, lr=2e-5, weight_decay=0.01, fused=fused)


def nonfinite_flag(opt, loss, check_grads=True):
    """0-dim f32 on the loss's device: 1 when the loss — or, with check_grads, any gradient the
    optimizer would apply — is NaN / Inf; MAX-reduced over the process group so every rank takes
    the same decision.  The gradient check is one multi-tensor inf-norm pass (no host sync); it
    catches an fp16 overflow in a backward whose loss stayed finite (the neck / heads run on one
    power-of-two gradient scale, ops.HeadScale)."""
    flag = (~torch.isfinite(loss.detach().reshape(-1)[0])).to(torch.float32)
    if check_grads:
        grads = [p.grad for g in opt.param_groups for p in g["params"] if p.grad is not None]
        if grads:
            norms = torch._foreach_norm(grads, float("inf"))
            bad = (~torch.isfinite(torch.stack([n.to(flag.device) for n in norms]))).any()
            flag = torch.maximum(flag, bad.to(torch.float32))
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if check_grads:  # an overflowed fp16 step re-primes the delayed gradient scales (ops.FP16_DELAYED_SCALE)
        from . import ops
        ops.watch_fp16_overflow(flag)
    return flag


def step_unless_nonfinite(opt, loss, check_grads=True):
    """opt.step(), skipped when the loss (or a gradient, check_grads) is NaN / Inf — the reference
    trainer skips such a step (train_denseclip.py:1323; e.g. a batch whose labels are all ignored
    gives a NaN CE).

    Fused torch optimizers take the decision ON THE DEVICE through their `found_inf` input (the
    AdamW kernel leaves parameters, moments and the step count untouched when it is non-zero): no
    host sync.  Non-fused optimizers read the flag on the host.  Either way the flag is
    MAX-reduced over the process group first, so every rank skips together and the replicas stay
    identical (a per-rank host check would let one rank skip while the others step)."""
    flag = nonfinite_flag(opt, loss, check_grads)
    if not all(g.get("fused") for g in opt.param_groups):
        if not bool(flag):
            opt.step()
        return
    opt.found_inf = flag
    try:
        opt.step()
    finally:
        del opt.found_inf


def train_step(model, opt, batch, silog=None, seg_weight=1.0, silog_weight=0.1):
    """One step: forward (DenseCLIP.forward train branch), loss, backward (DDP all-reduce
    overlapped with it), AdamW (skipped for a non-finite loss, step_unless_nonfinite).  Returns
    the loss tensor (no host sync)."""
    img, seg, depth, mask = batch
    out = model(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True)
    loss = loss_fn(out, seg, depth, mask, silog, seg_weight, silog_weight)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    # the gradients are checked too when the backward ran in fp16 (power-of-two scaled casts can
    # overflow there); bf16 / fp32 keep the reference's loss-only rule
    step_unless_nonfinite(opt, loss, check_grads=fp16_backward(model, img))
    return loss.detach()


class CapturedTrainStep:
    """train_step captured once into one HIP graph and replayed: forward, loss, backward, the
    non-finite check and the fused AdamW update (skipped on the device when the flag is set), and
    the refresh of the 16-bit weight copies the next forward reads — every launch of the step
    replayed from one hipGraphLaunch, so the host issues nothing per kernel and the step runs at
    the GPU's pace with the inter-kernel gaps of a graph (ops are stream-ordered and capture-safe:
    outputs from the caching allocator, no host synchronisation; the frozen text path becomes a
    parallel branch of the graph as in serve.CapturedForward).

    Call it with a batch of the captured shapes / dtypes (copied into the static input buffers)
    or with no argument (the same batch again); it returns the step's loss tensor (the SAME
    tensor every call).  Requirements: one process (no DDP: its bucketed all-reduce hooks are not
    captured here), a fused AdamW built with capturable=True (its step counts live on the device),
    and parameters that stay where they are.  An fp16 backward is captured with EXACT gradient
    scales (the delayed scales' use counter is host state, so ops takes exact scales under stream
    capture): its replays equal eager steps run with ops.FP16_DELAYED_SCALE = False bit for bit
    (tests/test_gpu_determinism.py; the step is bitwise reproducible since the fixed-order loss
    folds of ABI 7), and measured slower than the eager delayed-scale step (137.5 vs 135.1 ms,
    DESIGN.md §5), so the bench's fp16 line stays eager."""

    def __init__(self, model, opt, batch, silog=None, seg_weight=1.0, silog_weight=0.1, warmup=3):
        if isinstance(model, (torch.nn.parallel.DistributedDataParallel, GradAllReduce)):
            raise RuntimeError("CapturedTrainStep: one process only (the data-parallel all-reduce hooks are not captured)")
        if not all(g.get("fused") and g.get("capturable") for g in opt.param_groups):
            raise RuntimeError("CapturedTrainStep: needs a fused AdamW with capturable=True "
                               "(make_optimizer(..., capturable=True))")
        if not all(t.is_cuda for t in batch):
            raise RuntimeError("CapturedTrainStep: GPU batch tensors only (no CPU fallback)")
        self.static = [t.detach().clone() for t in batch]
        args = (silog, seg_weight, silog_weight)
        m = _unwrap(model)
        saved = getattr(m, "graph_text", None)
        if saved is not None:
            m.graph_text = "side"  # the text path as a forked branch of this capture (no nested graph)
        try:
            dev = self.static[0].device
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(max(1, warmup)):  # caches, allocator pools, the weight-refresh descriptor
                    train_step(model, opt, self.static, *args)
            torch.cuda.current_stream(dev).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.loss = train_step(model, opt, self.static, *args)
        finally:
            if saved is not None:
                m.graph_text = saved

    def __call__(self, batch=None):
        if batch is not None:
            for s, t in zip(self.static, batch):
                if s.shape != t.shape or s.dtype != t.dtype:
                    raise ValueError(f"CapturedTrainStep was captured for {tuple(s.shape)} {s.dtype}, "
                                     f"got {tuple(t.shape)} {t.dtype}")
                if s.data_ptr() != t.data_ptr():
                    s.copy_(t)
        self.graph.replay()
        return self.loss


def fp16_backward(model, img=None):
    """Whether the model's backward runs in fp16: 16-bit images set the compute dtype themselves
    (CLIPVisionTransformer._cdt), fp32 images use the backbone's compute_dtype."""
    if img is not None and img.dtype in (torch.bfloat16, torch.float16):
        return img.dtype == torch.float16
    bb = getattr(_unwrap(model), "backbone", None)
    return getattr(bb, "compute_dtype", None) == torch.float16


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
