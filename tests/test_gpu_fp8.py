"""fp8 attention forward (BASELINE config 5: "fp8 MFMA attention"); training runs the 16-bit
flash backward on the fp8 forward's (o, lse).

Two references per case:
  * an EMULATION of the kernel's arithmetic (torch.float8_e4m3fn rounding):
    q / k / v quantised with one scale per (image, head, q|k|v) = 448 / amax, the key sweep in
    64-key units with the running maximum, P rounded to e4m3 against the running maximum,
    l from the unrounded P.  Rounding to e4m3 is discontinuous: a P that the fp32 kernel and
    the float64 emulation put on opposite sides of a rounding midpoint (their scores differ by
    ~1e-6) moves by one e4m3 step (6-12 %), so a row dominated by two or three keys can land a
    few % off.  The kernel must therefore match the emulation to 5e-3 in the MEDIAN row (the
    16-bit output rounding; measured 0.02 % f16, 0.36 % bf16) and 2e-2 over all rows
    (measured <= 1.04 %).  lse is unaffected by P rounding but carries the MFMA's own dot-product
    error: v_mfma_scale_f32_32x32x64_f8f6f4 sums its 64 products to within ~2e-4 of the largest
    |product| (measured with N = 1, where lse is the score itself: tools/fp8_dot.py,
    profiles/r01ag_fp8_dot.log), i.e. not to fp32 precision, so lse is held to
    1e-3 + 5e-3 |lse|.  The packed e4m3 planes themselves are bit-exact against torch
    (tools/fp8_planes.py, profiles/r01ag_fp8_planes.log);
  * exact softmax attention on the same 16-bit inputs: the fp8 error itself, held to 1e-1.
    e4m3 carries 3 mantissa bits (relative rounding up to 6.25 %); on these inputs (score
    spread ~3 log2 units, a peaked softmax) the score error moves P by ~10 % and the output
    lands 6.5-8.5 % from exact (measured).  Through the whole ViT-B/16 model the maps and
    head outputs stay within 1.3 % of the fp32 reference (test_fp8_model_forward_vs_reference).
Both references run in float64 on the host.
"""
import math

import pytest
import torch

from helpers import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"
LOG2E = 1.4426950408889634


@pytest.fixture(autouse=True)
def _need(hip):
    torch.manual_seed(0)


def make_qkv(B, N, H, dt, spread=1.5):
    """16-bit qkv with q pre-multiplied by d^-0.5 log2(e) (the QKV GEMM epilogue's contract)."""
    C = 64 * H
    qkv = (torch.randn(B * N, 3 * C, device=DEV) * spread).to(dt)
    qkv[:, :C] = (qkv[:, :C].float() * (64 ** -0.5 * LOG2E)).to(dt)
    return qkv


def emulate(qkv, B, N, H, rows=None):
    """float64 on the host (a GPU fp32 GEMM may run at reduced internal precision); `rows`:
    the query rows to evaluate (every row is independent).  Returns o (B, len(rows), C) and
    lse (B, H, len(rows))."""
    C = 64 * H
    x = qkv.double().cpu().view(B, N, 3, H, 64)
    amax = x.abs().amax(dim=(1, 4))  # (B, 3, H)
    amax = torch.where(amax > 0, amax, torch.full_like(amax, 448.0))
    sc = (448.0 / amax).view(B, 1, 3, H, 1)
    x8 = (x * sc).clamp(-448, 448).float().to(torch.float8_e4m3fn).double()
    q8, k8, v8 = x8.permute(2, 0, 3, 1, 4)  # (B, H, N, 64)
    if rows is not None:
        q8 = q8[:, :, rows]
    R = q8.shape[2]
    d = amax / 448.0  # (B, 3, H)
    sscale = (d[:, 0] * d[:, 1]).view(B, H, 1, 1)
    dv = d[:, 2].view(B, H, 1, 1)
    m = torch.full((B, H, R, 1), -math.inf, dtype=torch.float64)
    l = torch.zeros(B, H, R, 1, dtype=torch.float64)
    acc = torch.zeros(B, H, R, 64, dtype=torch.float64)
    for u in range(0, N, 64):
        s = (q8 @ k8[:, :, u:u + 64].transpose(-1, -2)) * sscale
        mn = torch.maximum(m, s.amax(-1, keepdim=True))
        alpha = torch.exp2(m - mn)
        p = torch.exp2(s - mn)
        l = l * alpha + p.sum(-1, keepdim=True)
        acc = acc * alpha + p.float().to(torch.float8_e4m3fn).double() @ v8[:, :, u:u + 64]
        m = mn
    o = acc * dv / l
    return o.permute(0, 2, 1, 3).reshape(B, R, C), (m + torch.log2(l))[..., 0]


def exact(qkv, B, N, H, rows=None):
    C = 64 * H
    q, k, v = qkv.double().cpu().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    if rows is not None:
        q = q[:, :, rows]
    p = torch.softmax((q @ k.transpose(-1, -2)) / LOG2E, -1)  # q carries d^-0.5 log2(e)
    return (p @ v).permute(0, 2, 1, 3).reshape(B, q.shape[2], C)


def cls_split(N):
    """N = 1 + 256k: dclip_attn_fwd_fp8 computes query 0 (the CLS row) with the 16-bit
    split-key row pass of the bf16 forward, so that row is held to the EXACT attention (16-bit
    output rounding) instead of the fp8 emulation."""
    return N >= 257 and (N - 1) % 256 == 0


def check_row0_exact(o, lse, qkv, B, N, H):
    """o, lse: the kernel's row 0 (B, C) / (B, H) on the host in float64."""
    q, k, v = qkv.double().cpu().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = q[:, :, :1] @ k.transpose(-1, -2)  # (B, H, 1, N), log2 domain
    lref = torch.logsumexp(s * math.log(2.0), -1)[..., 0] / math.log(2.0)
    oref = (torch.softmax(s * math.log(2.0), -1) @ v)[:, :, 0].reshape(B, -1)
    assert rel_err(o, oref) < 1e-2, rel_err(o, oref)
    assert ((lse - lref).abs() <= 1e-3 + 1e-3 * lref.abs()).all(), float((lse - lref).abs().max())


def check_emulation(o, lse, ref, lref):
    assert rel_err(o, ref) < 2e-2, rel_err(o, ref)
    rows = ((o - ref).norm(dim=-1) / ref.norm(dim=-1).clamp(min=1e-30))
    assert float(rows.median()) < 5e-3, float(rows.median())
    assert ((lse - lref).abs() <= 1e-3 + 5e-3 * lref.abs()).all(), float((lse - lref).abs().max())


def pick(o, lse, B, N, H, rows):
    o = o.double().cpu().view(B, N, -1)[:, rows]
    return o, lse.double().cpu().view(B, H, N)[:, :, rows]


@pytest.mark.parametrize("N", [1, 2, 63, 64, 65, 129, 257, 1000, 2049])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_attn_fp8_matches_emulation_and_exact(N, dt):
    from denseclip_vit_multimodal_amd import ops
    B, H = 2, 3
    qkv = make_qkv(B, N, H, dt)
    o, lse = ops.attn_fwd_fp8(qkv, B, N, H)
    r0 = 1 if cls_split(N) else 0
    if r0:
        o0, l0 = pick(o, lse, B, N, H, torch.arange(1))
        check_row0_exact(o0[:, 0], l0[:, :, 0], qkv, B, N, H)
    rows = torch.arange(r0, N)
    o, lse = pick(o, lse, B, N, H, rows)
    ref, lref = emulate(qkv, B, N, H, rows)
    check_emulation(o, lse, ref, lref)
    e = rel_err(o, exact(qkv, B, N, H, rows))
    assert e < 1e-1, e


def test_attn_fp8_full_length_heads_and_batch():
    """The benchmark's sequence (N = 8193, 12 heads): per-(image, head) scales — a head scaled
    by 4x (scores x16) and an image scaled by 1/100 (uniform attention) come out as accurate as
    the rest."""
    from denseclip_vit_multimodal_amd import ops
    B, N, H = 2, 8193, 12
    qkv = make_qkv(B, N, H, torch.bfloat16).float().view(B, N, 3, H, 64)
    qkv[:, :, :, 5] *= 4.0
    qkv[1] *= 0.01
    qkv = qkv.view(B * N, -1).to(torch.bfloat16)
    o, lse = ops.attn_fwd_fp8(qkv, B, N, H)
    assert torch.isfinite(o).all()
    assert cls_split(N)
    o0, l0 = pick(o, lse, B, N, H, torch.arange(1))
    check_row0_exact(o0[:, 0], l0[:, :, 0], qkv, B, N, H)
    rows = torch.cat([torch.arange(1, 70), torch.randperm(N - 140)[:300] + 70, torch.arange(N - 70, N)])
    o, lse = pick(o, lse, B, N, H, rows)
    ref, lref = emulate(qkv, B, N, H, rows)
    ex = exact(qkv, B, N, H, rows)
    assert ((lse - lref).abs() <= 1e-3 + 5e-3 * lref.abs()).all()
    for b in range(B):
        for h in (0, 5, 11):
            sl = (b, slice(None), slice(64 * h, 64 * h + 64))
            check_emulation(o[sl], lse[b, h], ref[sl], lref[b, h])
            # head 5's scores are 16x larger, and so is their absolute e4m3 error (measured 27.8 %
            # from exact on image 0; the emulation check above still holds): fp8 attention is for
            # moderately peaked scores, as in the model test below
            assert rel_err(o[sl], ex[sl]) < (1e-1 if h != 5 else 3.5e-1), (b, h, rel_err(o[sl], ex[sl]))


def test_attn_fp8_spiky_scores():
    """A few dominant keys (the CLS-like spike): the running max moves mid-sweep."""
    from denseclip_vit_multimodal_amd import ops
    B, N, H = 1, 700, 2
    qkv = make_qkv(B, N, H, torch.bfloat16).float()
    C = 128
    qkv[[0, 350, 699], C:2 * C] *= 6.0
    qkv = qkv.to(torch.bfloat16)
    o, lse = ops.attn_fwd_fp8(qkv, B, N, H)
    o, lse = pick(o, lse, B, N, H, torch.arange(N))
    ref, lref = emulate(qkv, B, N, H)
    check_emulation(o, lse, ref, lref)
    assert rel_err(o, exact(qkv, B, N, H)) < 1e-1


def test_fp8_model_forward_vs_reference():
    """ViT-B/16 DenseCLIP (seg + depth heads) at 128x256 with every block's attention on the fp8
    kernel, against the reference's fp32 outputs (golden fixture): the fp8 error through 12
    blocks stays within 5e-2 on the maps, score map and head outputs (measured values are
    printed); the bf16-attention model is held to 1e-2 by test_gpu_parity."""
    from helpers import CITYSCAPES_CFG, CITYSCAPES_CLASSES, spec_state_dict, golden, images
    from denseclip_vit_multimodal_amd import DenseCLIP
    g = golden("vitb16_1x128x256")
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **CITYSCAPES_CFG)
    m.load_state_dict(spec_state_dict("cityscapes"))
    m.backbone.attn_fp8 = True
    m = m.to(DEV).eval()
    cap = {}
    m.backbone.register_forward_hook(lambda mod, i, o: cap.__setitem__("maps", [t.detach().float() for t in o]))
    m.decode_head.register_forward_hook(lambda mod, i, o: cap.__setitem__("seg", o.detach().float()))
    m.depth_head.register_forward_hook(lambda mod, i, o: cap.__setitem__("depth", o.detach().float()))
    with torch.no_grad():
        m(images(1, 128, 256).to(DEV).to(torch.bfloat16), return_loss=False)
    errs = {"map0": rel_err(cap["maps"][0], g["map0"]), "map11": rel_err(cap["maps"][11], g["map11"]),
            "seg_low": rel_err(cap["seg"], g["seg_low"]), "depth_low": rel_err(cap["depth"], g["depth_low"])}
    print("fp8 model errors", errs)
    for k, e in errs.items():
        assert e < 5e-2, (k, e)


def test_fp8_forward_bf16_backward_kernel():
    """Config 5 training: the fp8 forward's (o, lse) drive the 16-bit flash backward (P recomputed
    from the 16-bit q, k against the fp8 lse).  Against exact fp32 autograd the gradient carries
    the fp8 forward's error (o ~7 % off exact here); held to 1.5e-1 per q / k / v slice, and to
    the 16-bit backward's own tolerance against the same backward fed the exact forward's o / lse
    for dV (linear in P)."""
    from denseclip_vit_multimodal_amd import ops
    B, N, H = 2, 2049, 2
    C = 64 * H
    qkv = make_qkv(B, N, H, torch.bfloat16, spread=1.0)
    dout = torch.randn(B * N, C, device=DEV).to(torch.bfloat16)
    o8, l8 = ops.attn_fwd_fp8(qkv, B, N, H)
    dq8 = ops.attn_bwd(qkv, o8, dout, l8, B, N, H, 64 ** -0.5)
    assert torch.isfinite(dq8).all()
    ref = qkv.float().clone()
    ref[:, :C] /= (64 ** -0.5 * LOG2E)  # the unscaled q the 16-bit kernels' contract implies
    r = ref.clone().requires_grad_(True)
    q, k, v = r.view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    o = torch.softmax(q @ k.transpose(-1, -2) * 64 ** -0.5, -1) @ v
    o.permute(0, 2, 1, 3).reshape(B * N, C).backward(dout.float())
    errs = [rel_err(dq8[:, s].float(), r.grad[:, s]) for s in (slice(0, C), slice(C, 2 * C), slice(2 * C, 3 * C))]
    print("fp8-forward gradient errors vs exact (q, k, v)", errs)
    assert max(errs) < 1.5e-1, errs


def test_fp8_model_backbone_gradients():
    """ViT-B/16 widths, fp8 attention forward + 16-bit backward through all 12 blocks: backbone
    gradients of a linear functional of the maps against autograd through the fp32 oracle
    (bf16 attention is held to 2e-2 by test_gpu_parity)."""
    from helpers import CITYSCAPES_CFG, CITYSCAPES_CLASSES, spec_state_dict, images
    from oracle import denseclip_oracle as O
    from denseclip_vit_multimodal_amd import DenseCLIP
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **CITYSCAPES_CFG)
    m.load_state_dict(spec_state_dict("cityscapes"))
    bb = m.backbone.to(DEV).train()
    bb.attn_fp8 = True
    x = images(1, 128, 256)
    maps = bb(x.to(DEV).to(torch.bfloat16))
    gen = torch.Generator().manual_seed(5)
    ws = [torch.randn(mp.shape, generator=gen) for mp in maps]
    sum((mp.float() * w.to(DEV)).sum() for mp, w in zip(maps, ws)).backward()
    sd = {k: v.clone().requires_grad_(True) if k.startswith("backbone.") else v
          for k, v in spec_state_dict("cityscapes").items()}
    ref = O.vit_forward(x, sd, out_indices=list(range(12)))
    sum((r * w).sum() for r, w in zip(ref, ws)).backward()
    errs = {}
    for name, p in bb.named_parameters():
        if name == "proj":
            continue
        errs[name] = rel_err(p.grad, sd["backbone." + name].grad)
    worst = max(errs, key=errs.get)
    print("fp8 model gradient error: worst", worst, errs[worst], "median", sorted(errs.values())[len(errs) // 2])
    assert errs[worst] < 1.5e-1, (worst, errs[worst])
