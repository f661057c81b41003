"""The benchmark's own configuration (BASELINE configs[1]: ViT-B/16 DenseCLIP fwd+bwd, batch 8 @
1024x2048, bf16, mode F) checked in BACKWARD, plus the RCCL data-parallel path run for real.

  * attention at the headline shape (B = 8 images, H = 12 heads, N = 8193): forward and backward
    of sampled (image, head) slices against fp32 autograd, so the (b, h) indexing of the dQ,
    dK/dV and row-0 passes is checked where the bench runs them;
  * the whole ViT-B/16 backbone at B = 8: backbone gradients of a per-image linear functional of
    the 12 maps are the SUM of the same gradients taken one image at a time (images are
    independent in the ViT; the batched and single-image runs differ only in fp32 summation
    order of the weight gradients);
  * the bench's full train step (DenseCLIP, fused head losses, fused AdamW) at B = 8: finite loss
    and gradients, and the step's weight update reaches the next forward (the
    compute-dtype weight cache vs fused AdamW);
  * bench.py under torch.distributed.run with the "nccl" (RCCL) backend and DDP forced at world
    size 1: process-group init, DDP's bucketed all-reduce hooks and the HIP-graph text capture
    together on the GPU.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from helpers import CITYSCAPES_CFG, CITYSCAPES_CLASSES, TINY_CFG, images, rel_err, spec_state_dict
from test_gpu_kernels import prescale

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _need(hip):
    torch.manual_seed(0)


def test_attention_headline_shape_fwd_bwd():
    """B = 8, H = 12, N = 8193 (one launch of the bench's attention): sampled (b, h) slices of o,
    lse, dQ, dK, dV against fp32 autograd of that slice."""
    from denseclip_vit_multimodal_amd import ops
    B, H, N = 8, 12, 8193
    C = 64 * H
    qkv, qref = prescale(torch.randn(B * N, 3 * C, device=DEV).to(torch.bfloat16), H)
    dout = torch.randn(B * N, C, device=DEV).to(torch.bfloat16)
    o, lse = ops.attn_fwd(qkv, B, N, H, 64 ** -0.5)
    dqkv = ops.attn_bwd(qkv, o, dout, lse, B, N, H, 64 ** -0.5)
    assert torch.isfinite(dqkv).all() and torch.isfinite(o).all()
    for b, h in ((0, 0), (3, 7), (7, 11), (5, 2), (6, 6)):
        rows = slice(b * N, (b + 1) * N)
        cols = [slice(j * C + 64 * h, j * C + 64 * h + 64) for j in range(3)]
        q, k, v = (qref[rows, c].clone().requires_grad_(True) for c in cols)
        s = q @ k.t() * 0.125
        ref = torch.softmax(s, -1) @ v
        ref.backward(dout[rows, 64 * h:64 * h + 64].float())
        assert rel_err(o[rows, 64 * h:64 * h + 64].float(), ref) < 1.2e-2, (b, h)
        lref = torch.logsumexp(s, -1) / torch.log(torch.tensor(2.0))
        assert (lse.view(B, H, N)[b, h] - lref.detach()).abs().max() < 1e-2, (b, h)
        for name, c, g in zip("qkv", cols, (q.grad, k.grad, v.grad)):
            e = rel_err(dqkv[rows, c].float(), g)
            assert e < 4.8e-2, (b, h, name, e)
            # the CLS row (query 0 / key 0: the row-0 passes)
            e0 = float((dqkv[b * N, c].float() - g[0]).norm()) / max(float(g[0].norm()), 1e-3 * float(g.norm()))
            assert e0 < 4.8e-2, (b, h, name, "row 0", e0)


def _backbone():
    from denseclip_vit_multimodal_amd import DenseCLIP
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **CITYSCAPES_CFG)
    m.load_state_dict(spec_state_dict("cityscapes"))
    return m.backbone.to(DEV).train()


def test_vitb16_full_resolution_backward_is_additive_over_images():
    """ViT-B/16 at B = 8 x 1024x2048 (bf16, mode F backbone): d/dparams of sum_i <map_i, W_i>
    for the batch equals the sum over images of the same derivative taken image by image.

    Bound: bf16 rounding noise between two summation orders.  Measured in one process
    (tools/additivity_probe.py, profiles/r04/r06j_additivity.log): worst parameter class_embedding
    at 2.00e-3 with fp32 LayerNorm-backward inputs (the round-3 bound of 2e-3 sat on it) and
    2.34e-3 with the bf16 ones (ops.LN_DY_LP, one more bf16 rounding per element per block); the
    next parameters at 1.8e-3 either way."""
    bb = _backbone()
    B = 8
    x = images(B, 1024, 2048).to(DEV).to(torch.bfloat16)
    gen = torch.Generator(device=DEV).manual_seed(3)
    ws = [torch.randn(B, 768, 64, 128, device=DEV, generator=gen, dtype=torch.bfloat16) for _ in range(12)]

    def grads(sl):
        bb.zero_grad(set_to_none=True)
        maps = bb(x[sl].contiguous())
        sum((mp.float() * w[sl].float()).sum() for mp, w in zip(maps, ws)).backward()
        return {n: p.grad.detach().clone() for n, p in bb.named_parameters() if p.grad is not None}

    g_batch = grads(slice(0, B))
    assert len(g_batch) >= 12 * 12 and all(torch.isfinite(g).all() for g in g_batch.values())
    g_sum = None
    for i in range(B):
        gi = grads(slice(i, i + 1))
        g_sum = gi if g_sum is None else {k: g_sum[k] + gi[k] for k in g_sum}
    worst = max(((rel_err(g_batch[k], g_sum[k]), k) for k in g_batch))
    assert worst[0] < 3e-3, worst


def test_headline_train_step_two_steps():
    """The bench's step (DenseCLIP mode F, fused resize + CE / SILog, fused AdamW) at B = 8 x
    1024x2048 bf16: finite loss and gradients on every parameter that feeds the loss; the AdamW
    update of step 1 is what step 2's forward uses (cache refreshed, not stale)."""
    from denseclip_vit_multimodal_amd import ops
    from denseclip_vit_multimodal_amd.config import build_model, load_yaml
    from denseclip_vit_multimodal_amd.train import (freeze_for_mode, gradless_parameter_names, loss_fn,
                                                    make_optimizer, synth_batch)
    torch.manual_seed(0)
    m = build_model(load_yaml("denseclip_cityscapes.yaml"), clip_path_override="").to(DEV).train()
    m.fused_head_loss = True
    params = freeze_for_mode(m, "F")
    opt = make_optimizer(params)
    img, seg, depth, mask = synth_batch(8, 1024, 2048, torch.device(DEV))
    dead = set(gradless_parameter_names(m))
    losses = []
    for step in range(2):
        out = m(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True)
        loss = loss_fn(out, seg, depth, mask)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        losses.append(float(loss))
        for n, p in m.named_parameters():
            if p.requires_grad and n not in dead:
                assert p.grad is not None and torch.isfinite(p.grad).all(), (step, n)
        opt.step()
    assert all(torch.isfinite(torch.tensor(losses))), losses
    # the fused AdamW moved the fp32 masters without bumping their version counters; the
    # next forward must see the new weights: same output with a force-cleared cache
    w = m.backbone.transformer.resblocks[5].mlp.c_fc.weight
    cached = ops.WEIGHTS.get(w, torch.bfloat16)
    assert torch.equal(cached, w.detach().to(torch.bfloat16))
    m.eval()
    with torch.no_grad():
        a = m.backbone(img[:1])[-1].float()
        ops.invalidate_weight_cache()
        b = m.backbone(img[:1])[-1].float()
    assert torch.equal(a, b)


def _bench(args, nproc=1, port=29571, timeout=420):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", TORCH_DISTRIBUTED_DEBUG="DETAIL")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        print("---- bench stdout ----\n" + r.stdout[-4000:] + "\n---- bench stderr ----\n" + r.stderr[-8000:])
    assert r.returncode == 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("grad_dtype", ["fp32", "bf16"])
def test_bench_rccl_ddp_world_size_1(grad_dtype):
    """bench.py under torch.distributed.run with init_process_group("nccl") (RCCL) and the
    data-parallel wrapper forced at world size 1 (reference train_denseclip.py:1050-1054,
    utils.py:102-107): the timing barrier / max-reduce run through RCCL, and with bf16 gradients
    torch DDP's compressed bucket all-reduces (fp32: GradAllReduce, which skips the one-rank
    identity — its RCCL path is test_grad_allreduce_rccl_world_size_1); mode F at 512x1024."""
    line = _bench(["--ddp", "--grad-dtype", grad_dtype, "--steps", "2", "--warmup", "1", "--batch", "2",
                   "--height", "512", "--width", "1024", "--no-mode-r", "--cpu-baseline", "off"],
                  port=29571 if grad_dtype == "fp32" else 29572)
    assert line["config"]["ddp"] is True and line["config"]["grad_allreduce_dtype"] == grad_dtype
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["loss"] == line["loss"]  # finite, not NaN


def test_grad_allreduce_rccl_world_size_1():
    """train.GradAllReduce's RCCL path (coalesced and per-tensor in-place AVG all-reduces launched
    from the backward's post-accumulate-grad hooks, ~1 MB buckets) on a one-rank "nccl" group with
    the collectives issued: every bucket launched, the gradients those of the bare model
    (tests/rccl_allreduce_worker.py, in its own process)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29574",
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_allreduce_worker.py")], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print("---- stdout ----\n" + r.stdout[-4000:] + "\n---- stderr ----\n" + r.stderr[-8000:])
    assert r.returncode == 0
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["grads"] > 0 and res["buckets_coalesce_True"] > 1 and res["buckets_coalesce_False"] > 1, res
    assert res["hog_windows"] > 1, res


def test_bench_fp8_attention_trains():
    """BASELINE config 5: seg + depth train step with the fp8 attention forward (mode F)."""
    line = _bench(["--attn-fp8", "--steps", "2", "--warmup", "1", "--batch", "2", "--height", "512",
                   "--width", "1024", "--no-mode-r", "--cpu-baseline", "off"], port=29573)
    assert "e4m3" in line["dtype"] and line["roofline"]["launches"] > 0
    assert line["roofline_attn_fwd"]["launches"] > 0 and line["loss"] == line["loss"]
