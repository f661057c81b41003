"""Model-level parity of the HIP path against the reference (golden fixtures produced by the
reference itself) and the CPU oracle.

Tolerance (north star: "within 1e-3 relative fp16 tolerance"): with fp16 MFMA operands
and the fp32 residual stream / LayerNorm / softmax statistics, the norm-wise relative
error ||y - y_ref|| / ||y_ref|| of the maps, score map and pre-upsample logits must be
<= 1e-3 for the small fixtures; bf16 (the throughput dtype, 8 mantissa bits) is held to
1e-2.

Gradients.  The well-conditioned checks are in test_gpu_grad_parity.py (a linear functional of
the ViT-B/16 maps / heads at N = 129, 513 and 466, bounded by a 16-bit emulation's error).  The full tiny
train step (CE + SILog through train-mode BatchNorm, ReLU neck/heads at random init) is
ill-conditioned: perturbing the fp32 oracle's feature maps by 1e-3 relative noise moves
its own parameter gradients by 8-33 % element-wise (0.3 % in norm), so that step is held
to 3e-2 in every gradient NORM, and to 0.15 per tensor / 0.06 median on the sampled
elements — the fp16 HIP step lands at 5-8 % there, inside the reference's own noise band.
"""
import pytest
import torch
import torch.nn.functional as F

from helpers import (TINY_CFG, TINY_CTX_CFG, CITYSCAPES_CFG, VITL14_CFG, CITYSCAPES_CLASSES, spec_state_dict, golden, class_tokens,
                     images, rel_err, stats)

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _need(hip):
    pass


def build(name, cfg, cdt=torch.float16):
    from denseclip_vit_multimodal_amd import DenseCLIP
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **cfg)
    m.load_state_dict(spec_state_dict(name))
    m.backbone.compute_dtype = cdt
    return m.to(DEV).eval()


def capture(model):
    cap = {}
    model.decode_head.register_forward_hook(lambda m, i, o: cap.__setitem__("seg_low", o.detach().float()))
    model.depth_head.register_forward_hook(lambda m, i, o: cap.__setitem__("depth_low", o.detach().float()))
    model.backbone.register_forward_hook(lambda m, i, o: cap.__setitem__("maps", [t.detach().float() for t in o]))
    orig = model._process_features

    def wrapped(x):
        out = orig(x)
        cap["score"] = out[2].detach().float()
        cap["text"] = out[0].detach().float()
        return out
    model._process_features = wrapped
    return cap


@pytest.mark.parametrize("cdt,tol", [(torch.float16, 1e-3), (torch.bfloat16, 1e-2)])
def test_tiny_eval_vs_reference(cdt, tol):
    g = golden("tiny_eval")
    m = build("tiny", TINY_CFG, cdt)
    cap = capture(m)
    with torch.no_grad():
        out = m(g["input"].to(DEV), return_loss=False)
    for i in range(3):
        assert rel_err(cap["maps"][i], g[f"map{i}"]) < tol, i
    assert rel_err(cap["text"], g["text"]) < 1e-5
    assert rel_err(cap["score"], g["score"]) < tol
    assert rel_err(cap["seg_low"], g["seg_low"]) < tol
    assert rel_err(out["seg"], g["seg"]) < tol
    assert rel_err(out["depth"], g["depth"]) < tol


@pytest.mark.parametrize("cdt,tol", [(torch.float16, 1e-3), (torch.bfloat16, 1e-2)])
def test_vitb16_128x256_vs_reference(cdt, tol):
    g = golden("vitb16_1x128x256")
    m = build("cityscapes", CITYSCAPES_CFG, cdt)
    cap = capture(m)
    with torch.no_grad():
        out = m(images(1, 128, 256).to(DEV), return_loss=False)
    assert rel_err(cap["maps"][0], g["map0"]) < tol
    assert rel_err(cap["maps"][11], g["map11"]) < tol
    for i in range(12):
        fl = cap["maps"][i].flatten().cpu()
        assert rel_err(fl[g[f"map_idx{i}"]], g[f"map_val{i}"]) < 2 * tol, i
    assert rel_err(cap["score"], g["score"]) < tol
    assert rel_err(cap["seg_low"], g["seg_low"]) < tol
    assert rel_err(cap["depth_low"], g["depth_low"]) < tol
    assert rel_err(out["seg"].flatten().cpu()[g["seg_idx"]], g["seg_val"]) < tol


def test_vitb16_cfg1_2x512x1024_vs_reference():
    """BASELINE config 1 shape (N = 2049 tokens), fp16: the first and last read-out maps in full
    (2 x 768 x 32 x 64 each) within the north-star 1e-3, element samples of all 12 maps, the
    score map and both heads' pre-upsample outputs."""
    g = golden("vitb16_2x512x1024")
    m = build("cityscapes", CITYSCAPES_CFG, torch.float16)
    cap = capture(m)
    with torch.no_grad():
        m(images(2, 512, 1024).to(DEV), return_loss=False)
    errs = {}
    for i in (0, 11):
        mp = cap["maps"][i].cpu()
        assert mp.shape == g[f"map{i}"].shape
        errs[f"map{i}"] = rel_err(mp, g[f"map{i}"])
        # per image too (an indexing error confined to one image of the batch shows here)
        for b in range(2):
            errs[f"map{i}[{b}]"] = rel_err(mp[b], g[f"map{i}"][b])
        # and element-wise against the map's own scale
        errs[f"map{i} max|d|/max|ref|"] = float((mp - g[f"map{i}"]).abs().amax() / g[f"map{i}"].abs().amax())
    for k in ("seg_low", "depth_low", "score"):
        errs[k] = rel_err(cap[k], g[k])
    print({k: round(v, 6) for k, v in errs.items()})
    for k, v in errs.items():
        assert v < (3e-3 if "max|d|" in k else 1e-3), (k, v)
    for i in range(12):
        fl = cap["maps"][i].flatten().cpu()
        assert rel_err(fl[g[f"map_idx{i}"]], g[f"map_val{i}"]) < 2e-3, i
        assert torch.allclose(stats(cap["maps"][i].cpu()), g[f"map_stats{i}"], rtol=2e-3, atol=2e-3), i


def test_tiny_train_step_grads_vs_reference():
    """One full fine-tune step (every parameter trainable, BN in train mode, dropout off):
    loss and every parameter's gradient norm vs the reference's own step."""
    g = golden("tiny_train")
    m = build("tiny", TINY_CFG, torch.float16)
    m.train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()
    for p in m.parameters():
        p.requires_grad_(True)
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    x = g["input"].to(DEV)
    seg_t = g["seg_t"].to(DEV)
    out = m(x, gt_semantic_seg=seg_t, gt_depth=g["depth_t"].to(DEV), return_loss=True)
    ce = F.cross_entropy(out["main_output"], seg_t, ignore_index=255)
    sl = SILogLoss()(out["depth_output"], g["depth_t"].to(DEV), g["depth_m"].bool().to(DEV))
    loss = ce + 0.1 * sl
    assert abs(float(loss) - float(g["loss"][0])) < 2e-3 * float(g["loss"][0])
    loss.backward()
    params = dict(m.named_parameters())
    n = 0
    elem = []
    for k in g:
        if not k.startswith("gnorm/"):
            continue
        name = k[len("gnorm/"):]
        gr = params[name].grad
        assert gr is not None, name
        ref_norm = float(g[k])
        assert abs(float(gr.double().norm()) - ref_norm) <= 3e-2 * ref_norm + 1e-6, name
        vals = gr.flatten().cpu()[g["gidx/" + name]]
        e = rel_err(vals, g["gval/" + name])
        # conditioning-limited bound (module docstring): the fp32 oracle's own gradients move
        # 8-33 % element-wise under a 1e-3 relative perturbation of the feature maps
        assert e < 0.15, (name, e)
        elem.append(e)
        n += 1
    assert n == sum(1 for k in g if k.startswith("gnorm/")) and n >= 60, n  # every golden parameter
    elem.sort()
    assert elem[len(elem) // 2] < 0.06, elem[len(elem) // 2]


@pytest.mark.parametrize("cdt,tol", [(torch.float16, 1e-3), (torch.bfloat16, 1e-2)])
def test_vitl14_120x230_vs_reference(cdt, tol):
    """BASELINE config 4's architecture (ViT-L/14, 24 layers x 16 heads, patch 14) against the
    reference at 120x230 (not a multiple of 14: floor grid 8x16, N = 129)."""
    g = golden("vitl14_1x120x230")
    m = build("vitl14", VITL14_CFG, cdt)
    cap = capture(m)
    with torch.no_grad():
        out = m(images(1, 120, 230).to(DEV), return_loss=False)
    assert rel_err(cap["maps"][0], g["map0"]) < tol
    assert rel_err(cap["maps"][3], g["map3"]) < tol
    for i in range(4):
        fl = cap["maps"][i].flatten().cpu()
        assert rel_err(fl[g[f"map_idx{i}"]], g[f"map_val{i}"]) < 2 * tol, i
    assert rel_err(cap["score"], g["score"]) < tol
    assert rel_err(cap["seg_low"], g["seg_low"]) < tol
    assert rel_err(cap["depth_low"], g["depth_low"]) < tol
    assert rel_err(out["seg"].flatten().cpu()[g["seg_idx"]], g["seg_val"]) < tol


def test_vitl14_full_resolution_train_step():
    """ViT-L/14 at 1024x2048 (grid 73x146, N = 10659 = 1 + 64*166 + 34: the ragged-N attention
    kernels): one bf16 fwd+bwd on one image gives finite backbone gradients, and the eval
    forward of the same image is per-image independent within a batch of two."""
    m = build("vitl14", VITL14_CFG, torch.bfloat16)
    m.train()
    for p in m.parameters():
        p.requires_grad_(True)
    x = images(2, 1024, 2048).to(DEV).to(torch.bfloat16)
    seg_t = torch.randint(0, 19, (1, 1024, 2048), device=DEV)
    o = m(x[:1].contiguous(), gt_semantic_seg=seg_t, return_loss=True)
    assert o["main_output"].shape == (1, 19, 1024, 2048)
    F.cross_entropy(o["main_output"], seg_t, ignore_index=255).backward()
    for name in ("conv1.weight", "transformer.resblocks.0.attn.in_proj_weight",
                 "transformer.resblocks.23.mlp.c_proj.weight"):
        gr = dict(m.backbone.named_parameters())[name].grad
        assert gr is not None and torch.isfinite(gr).all() and gr.abs().sum() > 0, name
    m.eval()
    cap = capture(m)
    with torch.no_grad():
        m(x, return_loss=False)
        seg2 = cap["seg_low"].clone()
        assert cap["maps"][0].shape == (2, 1024, 73, 146)
        m(x[1:].contiguous(), return_loss=False)
        seg1 = cap["seg_low"]
    assert torch.isfinite(seg2).all()
    assert rel_err(seg2[1:], seg1) < 1e-2


def test_full_resolution_properties():
    """1024x2048 (N = 8193, the benchmark shape): too large for the oracle in a test, so
    size-independent properties: finite outputs, per-image independence inside a batch
    (image 1 of a batch of 2 == the same image alone), and the final resize equals the
    HIP bilinear of the head output."""
    m = build("cityscapes", CITYSCAPES_CFG, torch.bfloat16)
    x = images(2, 1024, 2048).to(DEV).to(torch.bfloat16)
    cap = capture(m)
    with torch.no_grad():
        out2 = m(x, return_loss=False)
        seg_low2 = cap["seg_low"].clone()
        m(x[1:].contiguous(), return_loss=False)
        seg_low1 = cap["seg_low"]
    assert out2["seg"].shape == (2, 19, 1024, 2048)
    assert torch.isfinite(out2["seg"]).all()
    assert rel_err(seg_low2[1:], seg_low1) < 1e-2
    ref = F.interpolate(seg_low2, size=(1024, 2048), mode="bilinear", align_corners=False)
    assert rel_err(out2["seg"], ref) < 1e-2


@pytest.mark.parametrize("img_dtype", [torch.float32, torch.bfloat16])
def test_fused_head_loss_matches_materialised(img_dtype):
    """fused_head_loss (resize + CE / SILog in one kernel each) gives the loss and every
    parameter gradient of the reference formulation (materialised resize, F.cross_entropy,
    SILogLoss) on the same model and batch."""
    from denseclip_vit_multimodal_amd.train import loss_fn, synth_batch
    torch.manual_seed(0)
    m = build("tiny", TINY_CFG, torch.bfloat16)
    m.train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()
    for p in m.parameters():
        p.requires_grad_(True)
    img, seg, depth, mask = synth_batch(2, 64, 128, DEV, image_dtype=img_dtype)
    res = []
    for fused in (False, True):
        m.fused_head_loss = fused
        m.zero_grad(set_to_none=True)
        out = m(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True)
        loss = loss_fn(out, seg, depth, mask)
        loss.backward()
        res.append((float(loss), {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}))
    (l0, g0), (l1, g1) = res
    assert abs(l0 - l1) < 1e-4 * abs(l0), (l0, l1)
    assert g0.keys() == g1.keys() and len(g0) > 20
    for k in g0:
        # heads / neck: the two formulations agree to fp32 rounding; behind them the bf16 ViT
        # backward re-rounds a ~1e-6 different input gradient (module docstring: ill-conditioned)
        assert rel_err(g1[k], g0[k]) < (2e-2 if k.startswith("backbone.") else 2e-3), k


def test_text_path_graph_replay_matches_eager():
    """The frozen text path replayed from its captured HIP graph gives the eager result, is
    recomputed on every replay (a changed context token changes it), and a trainable text
    parameter falls back to eager execution."""
    m = build("tiny", TINY_CFG, torch.bfloat16)
    for p in m.text_encoder.parameters():
        p.requires_grad_(False)
    if m.contexts is not None:
        m.contexts.requires_grad_(False)
    dev = torch.device(DEV)
    m.graph_text = False
    eager = m._text_embeddings(2, dev).clone()
    m.graph_text = True
    g1 = m._text_embeddings(2, dev).clone()
    g2 = m._text_embeddings(2, dev).clone()
    assert m._text_graph is not None
    assert torch.allclose(g1, eager, rtol=1e-5, atol=1e-6) and torch.equal(g1, g2)
    if m.contexts is not None:
        with torch.no_grad():
            m.contexts.add_(0.5)  # in place: same storage, the graph reads the new values
        g3 = m._text_embeddings(2, dev).clone()
        m.graph_text = False
        assert not torch.equal(g3, g1)
        assert torch.allclose(g3, m._text_embeddings(2, dev), rtol=1e-5, atol=1e-6)
        m.graph_text = True
    m.text_encoder.text_projection.requires_grad_(True)
    graph_before = m._text_graph
    m._text_embeddings(2, dev)
    assert m._text_graph is graph_before  # eager path taken: no new capture, no replay needed


def test_text_prelaunch_on_side_stream_matches_in_line():
    """The forward replays the captured text graph on a side stream before the backbone
    (DenseCLIP._text_prelaunch) and the score branch waits for it: the same class embeddings and
    score map as the golden reference, the pending replay is consumed, and an in-place context
    update between forwards is seen by the prelaunched replay."""
    g = golden("tiny_ctx_eval")
    m = build("tiny_ctx", TINY_CTX_CFG, torch.float16)
    for p in list(m.text_encoder.parameters()) + [m.contexts]:
        p.requires_grad_(False)
    cap = capture(m)
    x = g["input"].to(DEV)
    with torch.no_grad():
        m(x, return_loss=False)  # captures the graph in line
        assert m._text_graph is not None
        t1 = cap["text"].clone()
        m(x, return_loss=False)  # prelaunched replay
        assert getattr(m, "_text_pending", None) is None
        assert torch.equal(cap["text"], t1)
        assert rel_err(cap["text"].cpu(), g["text"]) < 1e-3
        assert rel_err(cap["score"].cpu(), g["score"]) < 1e-3
        m.contexts.add_(0.25)
        m(x, return_loss=False)
        t3 = cap["text"].clone()
        m.graph_text = False
        m(x, return_loss=False)
    assert not torch.equal(t3, t1)
    assert rel_err(t3, cap["text"]) < 1e-3


@pytest.mark.parametrize("graph_text", [False, True])
def test_tiny_context_decoder_vs_reference(graph_text):
    """The ContextDecoder branch on the GPU (text path and decoder in torch, ViT / projections /
    score map on the HIP kernels) against the reference's context-fused class embeddings and
    score map."""
    g = golden("tiny_ctx_eval")
    m = build("tiny_ctx", TINY_CTX_CFG, torch.float16)
    if graph_text:
        for p in list(m.text_encoder.parameters()) + [m.contexts]:
            p.requires_grad_(False)
    cap = capture(m)
    with torch.no_grad():
        m(g["input"].to(DEV), return_loss=False)
    assert rel_err(cap["text"].cpu(), g["text"]) < 1e-3
    assert rel_err(cap["score"].cpu(), g["score"]) < 1e-3
    assert rel_err(cap["seg_low"].cpu(), g["seg_low"]) < 1e-3


def test_ddp_two_ranks_one_gpu_graphed_text_path():
    """DDP train steps (gloo, 2 ranks sharing the GPU) with fused losses and the HIP-graph text
    path: the capture coexists with the communication threads and the ranks stay in sync."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29561",
                        os.path.join(root, "tools", "ddp_gpu_check.py")],
                       cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "parameters identical across ranks: True" in r.stdout


@pytest.mark.parametrize("img", ["fp32", "bf16"])
def test_ddp_two_ranks_mode_f_gradients_match_single_process(img):
    """mode F DDP (ViT BlockFn backward, HIP neck / heads; gloo, 2 ranks on the
    GPU) — every post-all-reduce gradient equals the single-process average of the two shards'
    gradients (per-rank BatchNorm, as in the reference), and the ranks agree."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29563" if img == "fp32" else "29564",
                        os.path.join(root, "tools", "ddp_gpu_check.py"), "--grads", "--img", img],
                       cwd=root, env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout[-1500:])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "grads check ok: True" in r.stdout


@pytest.mark.parametrize("fp8", [False, True])
def test_captured_forward_matches_eager(fp8):
    """serve.CapturedForward (the eval forward replayed from one HIP graph, the text path captured
    inline) gives the eager forward's seg / depth bit for bit, for new inputs copied into the
    captured buffer, and refuses another input shape."""
    from denseclip_vit_multimodal_amd.serve import CapturedForward
    m = build("cityscapes", CITYSCAPES_CFG, torch.bfloat16)
    m.backbone.attn_fp8 = fp8
    x1 = images(2, 256, 512, seed=1).to(DEV).to(torch.bfloat16)
    x2 = images(2, 256, 512, seed=2).to(DEV).to(torch.bfloat16)
    with torch.no_grad():
        e1 = {k: v.clone() for k, v in m(x1, return_loss=False).items()}
        e2 = {k: v.clone() for k, v in m(x2, return_loss=False).items()}
    cf = CapturedForward(m, x1)
    assert m.graph_text  # restored after the capture
    for x, e in ((x2, e2), (x1, e1), (x2, e2)):
        out = cf(x)
        torch.cuda.synchronize()
        for k in ("seg", "depth"):
            assert torch.equal(out[k], e[k]), k
    with pytest.raises(ValueError):
        cf(x1[:1])


def test_captured_train_step_matches_eager():
    """train.CapturedTrainStep (forward + loss + backward + the non-finite check + fused AdamW + the
    16-bit weight-copy refresh replayed from one HIP graph) takes the same steps as eager
    train_step from the same start: two bf16 models built from one seed (dropout off, so both arms
    draw nothing at random), five eager steps against three warm-up steps + two replays — losses
    and every parameter within fp32 rounding, and the replays see new batches copied into the
    captured buffers.  Refuses a non-capturable optimizer."""
    import torch.nn as nn
    from denseclip_vit_multimodal_amd import DenseCLIP
    from denseclip_vit_multimodal_amd.train import CapturedTrainStep, freeze_for_mode, make_optimizer, synth_batch, \
        train_step

    def make():
        torch.manual_seed(0)
        m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **TINY_CTX_CFG).to(DEV).train()
        m.backbone.compute_dtype = torch.bfloat16
        for mod in m.modules():
            if isinstance(mod, nn.Dropout):
                mod.p = 0.0
        return m, make_optimizer(freeze_for_mode(m, "F"), capturable=True)

    b1 = synth_batch(2, 128, 256, torch.device(DEV), 0, image_dtype=torch.bfloat16)
    b2 = synth_batch(2, 128, 256, torch.device(DEV), 1, image_dtype=torch.bfloat16)
    ma, oa = make()
    la = [float(train_step(ma, oa, b)) for b in (b1, b1, b1, b2, b1)]
    mb, ob = make()
    with pytest.raises(RuntimeError):
        CapturedTrainStep(mb, make_optimizer([p for p in mb.parameters() if p.requires_grad]), b1)
    cap = CapturedTrainStep(mb, ob, b1)  # three eager warm-up steps on b1
    lb = [float(cap(b2)), float(cap(b1))]
    torch.cuda.synchronize()
    for x, y in zip(lb, la[3:]):
        assert abs(x - y) <= 1e-5 * abs(y), (lb, la)
    pa = dict(ma.named_parameters())
    for n, p in mb.named_parameters():
        ref = pa[n].detach()
        d = float((p.detach() - ref).abs().max())
        assert d <= 1e-5 * max(float(ref.abs().max()), 1e-30), (n, d)
