"""fp16 training path: the power-of-two gradient scale is computed ON THE DEVICE
(dclip_grad_scale) and read by the cast / token / GEMM kernels through a pointer, so an fp16
backward makes no device->host round trip.  The scaled ops must equal the
same ops with the scale passed as a host float (bit-exact: a power-of-two factor)."""
import math

import pytest
import torch

from helpers import CITYSCAPES_CFG, CITYSCAPES_CLASSES, images, rel_err, spec_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _need(hip):
    pass


def host_scale(g, target=16.0):
    """The formula dclip_grad_scale restates (include/dclip.h)."""
    amax = float(g.abs().amax())
    if not math.isfinite(amax) or amax == 0.0:
        return 1.0
    return 2.0 ** max(-60, min(60, math.floor(math.log2(target / amax))))


@pytest.mark.parametrize("mag,n", [(1e-7, 1 << 20), (3.0, 4099), (1e-30, 77), (1e30, 1000), (1e-9, 8 * 8193 * 768)])
def test_grad_scale_matches_host_formula(mag, n):
    from denseclip_vit_multimodal_amd import ops
    g = torch.randn(n, device=DEV) * mag
    g[-1] = 40 * mag  # the maximum in the ragged tail (n % 4 != 0 for two cases)
    ws = ops.grad_scale(g, torch.float16).cpu()
    s = host_scale(g)
    assert ws.tolist() == [s, 1.0 / s, 0.0, 0.0]
    assert ops.grad_scale(g, torch.bfloat16) is None  # bf16 has the fp32 exponent range


@pytest.mark.parametrize("bad", [0.0, float("inf"), float("nan")])
def test_grad_scale_degenerate_is_one(bad):
    from denseclip_vit_multimodal_amd import ops
    g = torch.zeros(1000, device=DEV) if bad == 0.0 else torch.randn(1000, device=DEV)
    g[123] = bad
    assert ops.grad_scale(g, torch.float16).cpu().tolist() == [1.0, 1.0, 0.0, 0.0]


@pytest.mark.parametrize("bdt", [torch.float16, torch.float32])
@pytest.mark.parametrize("rows,ntok,with_scale", [(2 * 513, 513, True), (8 * 8193, 8193, True), (3 * 65, 65, False)])
def test_add_readout_amax(bdt, rows, ntok, with_scale):
    """dclip_add_readout_amax (the fp16 backward's read-out fold): sum = a + b * (1/s of a HeadScale
    pair) with b's CLS rows masked, bitwise as torch computes it, and the grad_scale pair of the
    sum (the host formula); the workspace protocol leaves the pair reusable."""
    from denseclip_vit_multimodal_amd import ops
    cols = 768
    a = torch.randn(rows, cols, device=DEV) * 1e-6
    b = (torch.randn(rows, cols, device=DEV) * 8).to(bdt)
    b[ntok + 3, 5] = 4000.0  # the maximum, in a non-CLS row
    b[0, 7] = 1e30 if bdt == torch.float32 else 6e4  # CLS rows are ignored, maximum or not
    hs = torch.tensor([2.0 ** 20, 2.0 ** -20, 0.0, 0.0], device=DEV) if with_scale else None
    sm, ws = ops.D().add_readout_amax(a, b, ntok, hs, ops.FP16_GRAD_AMAX)
    keep = (torch.arange(rows, device=DEV) % ntok != 0)[:, None]
    bs = b.float() * (hs[1] if with_scale else 1.0)
    ref = torch.where(keep, a + bs, a)
    assert torch.equal(sm, ref)
    s = host_scale(ref)
    assert ws.cpu().tolist() == [s, 1.0 / s, 0.0, 0.0]
    assert torch.equal(ops.grad_scale(sm, torch.float16), ws)  # same pair as the separate pass


def _ds_state(prev_scale):
    """A DelayedScale seeded as after an exact cast with scale prev_scale (dclip.h's seeding rule)."""
    from denseclip_vit_multimodal_amd import ops
    ds = ops.DelayedScale()
    ds.prime(0, torch.tensor([prev_scale, 1.0 / prev_scale, 0.0, 0.0], device=DEV))
    return ds


@pytest.mark.parametrize("with_b", [True, False])
@pytest.mark.parametrize("rows,ntok", [(2 * 513, 513), (8 * 8193, 8193)])
def test_add_readout_cast_scaled(rows, ntok, with_b):
    """The delayed-scale fold: sum as dclip_add_readout_amax computes it (bitwise), lp = (f16)(sum *
    s) with s the previous use's scale (bitwise: a power of two), the pair it used; the NEXT call
    casts with THIS sum's exact scale (the host formula), and so on (three calls: the state's
    shards rotate through all three slots)."""
    from denseclip_vit_multimodal_amd import ops
    cols = 768
    a = torch.randn(rows, cols, device=DEV) * 1e-6
    b = (torch.randn(rows, cols, device=DEV) * 8).half() if with_b else None
    hs = torch.tensor([2.0 ** 20, 2.0 ** -20, 0.0, 0.0], device=DEV)
    ds = _ds_state(2.0 ** 17)
    keep = (torch.arange(rows, device=DEV) % ntok != 0)[:, None]
    s_expect = 2.0 ** 17
    for it in range(4):
        ai = a * 4.0 ** it
        sm, lp, pair = ops.add_readout_cast_scaled(ai, b, ntok, hs if with_b else None, ds, 0)
        r = torch.where(keep, ai + b.float() * hs[1], ai) if with_b else ai
        if with_b:
            assert torch.equal(sm, r)
        assert torch.equal(lp, (r * s_expect).half()), it
        assert pair[:2].cpu().tolist() == [s_expect, 1.0 / s_expect], it
        s_expect = host_scale(r)


def test_delayed_scale_keeps_scale_on_nonfinite_or_zero():
    """A previous maximum that is not finite (an inf from an overflow upstream) or zero (an unused
    gradient) says nothing about the site's range: the next call keeps the previous call's scale."""
    from denseclip_vit_multimodal_amd import ops
    ds = _ds_state(2.0 ** 12)
    bad = torch.randn(4 * 65, 768, device=DEV) * 1e-3
    bad[7, 9] = float("inf")
    _, _, p1 = ops.add_readout_cast_scaled(bad, None, 65, None, ds, 0)
    _, _, p2 = ops.add_readout_cast_scaled(torch.zeros_like(bad), None, 65, None, ds, 0)
    _, _, p3 = ops.add_readout_cast_scaled(bad.nan_to_num(posinf=0.0), None, 65, None, ds, 0)
    for p in (p1, p2, p3):
        assert p[:2].cpu().tolist() == [2.0 ** 12, 2.0 ** -12]


@pytest.mark.parametrize("cols", [768, 1024])
def test_layernorm_bwd_scaled(cols):
    """dclip_layernorm_bwd_scaled == layernorm_bwd (dx, dw, db) plus lp = (f16)(dx * s) on the
    previous use's scale, the pair; the next call casts with this dx's exact scale."""
    from denseclip_vit_multimodal_amd import ops
    rows = 8 * 1025
    x = torch.randn(rows, cols, device=DEV)
    w = torch.rand(cols, device=DEV) + 0.5
    b = torch.randn(cols, device=DEV)
    _, mean, rstd = ops.layernorm_fwd(x, w, b, torch.float16)
    dy = torch.randn(rows, cols, device=DEV) * 1e-7
    res = torch.randn(rows, cols, device=DEV) * 1e-7
    dw0, db0 = torch.zeros(cols, device=DEV), torch.zeros(cols, device=DEV)
    dx0 = ops.layernorm_bwd(dy, x, w, mean, rstd, dw0, db0, res=res)
    ds = _ds_state(2.0 ** 21)
    s_expect = 2.0 ** 21
    for it in range(2):
        dw1, db1 = torch.zeros(cols, device=DEV), torch.zeros(cols, device=DEV)
        dx1, lp, pair = ops.layernorm_bwd_scaled(dy, x, w, mean, rstd, dw1, db1, res, ds, 0)
        # the two instantiations may contract the row formula's multiply-adds differently: ulps
        assert rel_err(dx1, dx0) < 1e-6
        assert rel_err(dw1, dw0) < 1e-6 and rel_err(db1, db0) < 1e-6  # atomics: order-dependent sums
        assert torch.equal(lp, (dx1 * s_expect).half())
        assert pair[:2].cpu().tolist() == [s_expect, 1.0 / s_expect]
        s_expect = host_scale(dx1)


@pytest.mark.parametrize("cols", [768, 1024])
@pytest.mark.parametrize("form", ["res", "lp", "scaled", "scaled_add"])
def test_layernorm_bwd_f16_dy_on_scale(cols, form):
    """ABI 6: an fp16 dy still on its gradient scale s, read as dy * 1/s (dy_scale = the (s, 1/s)
    pair) by every LN backward form the fp16 block uses == the same form on the fp32 dy * 1/s
    (bitwise: one fp32 multiply either way, the rest the same instruction stream)."""
    from denseclip_vit_multimodal_amd import ops
    rows, ntok = 4 * 257, 257
    x = torch.randn(rows, cols, device=DEV)
    w = torch.rand(cols, device=DEV) + 0.5
    b = torch.randn(cols, device=DEV)
    _, mean, rstd = ops.layernorm_fwd(x, w, b, torch.float16)
    s = 2.0 ** 22
    pair = torch.tensor([s, 1.0 / s, 0.0, 0.0], device=DEV)
    dyh = (torch.randn(rows, cols, device=DEV) * 1e-6 * s).half()  # scaled: a 16-magnitude fp16 operand
    dyf = dyh.float() * pair[1]
    res = torch.randn(rows, cols, device=DEV) * 1e-6
    add = (torch.randn(rows, cols, device=DEV) * 8).half()
    out = []
    for dy, sc in ((dyf, None), (dyh, pair)):
        dw, db = torch.zeros(cols, device=DEV), torch.zeros(cols, device=DEV)
        if form == "res":
            r = (ops.layernorm_bwd(dy, x, w, mean, rstd, dw, db, res=res, dy_scale=sc),)
        elif form == "lp":
            r = ops.layernorm_bwd(dy, x, w, mean, rstd, dw, db, res=res, lp_dtype=torch.float16, dy_scale=sc)
        elif form == "scaled":
            r = ops.layernorm_bwd_scaled(dy, x, w, mean, rstd, dw, db, res, _ds_state(2.0 ** 17), 0, dy_scale=sc)
        else:
            r = ops.layernorm_bwd_scaled_add(dy, x, w, mean, rstd, dw, db, res, add, ntok, pair, _ds_state(2.0 ** 17),
                                             0, dy_scale=sc)
        r = tuple(r)
        if form in ("scaled", "scaled_add"):
            r = r[:2] + (r[2][:2],)  # the pair: (s, 1/s) are written, its other two floats are not
        out.append(r + (dw, db))
    for a, c in zip(*out):
        assert torch.equal(a, c)


def test_layernorm_bwd_dy_ntok_masks_cls_rows():
    """dy_ntok: a token-buffer gradient whose CLS rows (row % ntok == 0) hold garbage reads them as
    0 — the ln_post read-out's backward straight from the neck's 16-bit gradient buffer (bitwise the
    fp32 copy with the CLS rows zeroed and the heads' 1/s multiplied in, the path it replaces)."""
    from denseclip_vit_multimodal_amd import ops
    rows, cols, ntok = 3 * 129, 768, 129
    x = torch.randn(rows, cols, device=DEV)
    w = torch.rand(cols, device=DEV) + 0.5
    b = torch.randn(cols, device=DEV)
    _, mean, rstd = ops.layernorm_fwd(x, w, b, torch.float16)
    hs = torch.tensor([2.0 ** 10, 2.0 ** -10, 0.0, 0.0], device=DEV)
    g = torch.randn(rows, cols, device=DEV).half()
    g.view(3, ntok, cols)[:, 0] = float("nan")  # never read
    ref = g.float()
    ref.view(3, ntok, cols)[:, 0].zero_()
    ref.mul_(hs[1])
    dw0, db0 = torch.zeros(cols, device=DEV), torch.zeros(cols, device=DEV)
    dx0 = ops.layernorm_bwd(ref, x, w, mean, rstd, dw0, db0)
    dw1, db1 = torch.zeros(cols, device=DEV), torch.zeros(cols, device=DEV)
    dx1 = ops.layernorm_bwd(g, x, w, mean, rstd, dw1, db1, dy_scale=hs, dy_ntok=ntok)
    assert torch.equal(dx1, dx0) and torch.equal(dw1, dw0) and torch.equal(db1, db0)


@pytest.mark.parametrize("adt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("with_scale", [True, False])
def test_layernorm_bwd_scaled_add(adt, with_scale):
    """dclip_layernorm_bwd_scaled_add (the fp16 read-out fold: ln_1 backward of the next block +
    the map gradient times the heads' 1/s, CLS rows masked, + the fp16 operand on the map block's
    delayed scale) == layernorm_bwd then the add (dx within ulps: another instantiation may contract
    the multiply-adds differently), lp = (f16)(dx * s) with the previous use's scale (bitwise), the
    pair; the next call casts with this dx's exact scale."""
    from denseclip_vit_multimodal_amd import ops
    rows, cols, ntok = 4 * 257, 768, 257
    x = torch.randn(rows, cols, device=DEV)
    w = torch.rand(cols, device=DEV) + 0.5
    b = torch.randn(cols, device=DEV)
    _, mean, rstd = ops.layernorm_fwd(x, w, b, torch.float16)
    dy = torch.randn(rows, cols, device=DEV) * 1e-7
    res = torch.randn(rows, cols, device=DEV) * 1e-7
    add = (torch.randn(rows, cols, device=DEV) * 8).to(adt)
    hs = torch.tensor([2.0 ** 20, 2.0 ** -20, 0.0, 0.0], device=DEV) if with_scale else None
    dw0, db0 = torch.zeros(cols, device=DEV), torch.zeros(cols, device=DEV)
    dx0 = ops.layernorm_bwd(dy, x, w, mean, rstd, dw0, db0, res=res)
    keep = (torch.arange(rows, device=DEV) % ntok != 0)[:, None]
    ref = torch.where(keep, dx0 + add.float() * (hs[1] if with_scale else 1.0), dx0)
    ds = _ds_state(2.0 ** 17)
    s_expect = 2.0 ** 17
    for it in range(2):
        dw1, db1 = torch.zeros(cols, device=DEV), torch.zeros(cols, device=DEV)
        dx1, lp, pair = ops.layernorm_bwd_scaled_add(dy, x, w, mean, rstd, dw1, db1, res, add, ntok, hs, ds, 0)
        assert rel_err(dx1, ref) < 1e-6
        assert rel_err(dw1, dw0) < 1e-6 and rel_err(db1, db0) < 1e-6  # atomics: order-dependent sums
        assert torch.equal(lp, (dx1 * s_expect).half()), it
        assert pair[:2].cpu().tolist() == [s_expect, 1.0 / s_expect], it
        s_expect = host_scale(dx1)


def test_fp16_readout_grad_fold_matches_unfolded():
    """ViT-B/16 backbone + fusion neck in fp16 with delayed scales: a first backward primes every
    block's scales (no fold: a site's first cast is exact), the second folds each read-out map's
    gradient into the next block's ln_1 backward on the map block's delayed scale
    (dclip_layernorm_bwd_scaled_add).  Its gradients equal the unfolded path's within the 16-bit
    noise floor: the two LN instantiations may round dx an ulp apart, and such ulps re-rounded
    through every fp16 cast of the backward move gradients by ~1e-3 — measured in one process
    (tools/fold_fp16_probe.py, profiles/r04/r06o_fold_probe.log): fold on vs off 9.9e-4 worst
    parameter, the output gradient scaled by (1 + 2^-20) 3.4e-3, a repeat 4e-8."""
    from denseclip_vit_multimodal_amd import DenseCLIP
    from denseclip_vit_multimodal_amd import ops as O
    from helpers import CITYSCAPES_CFG, CITYSCAPES_CLASSES, images, spec_state_dict
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **CITYSCAPES_CFG)
    m.load_state_dict(spec_state_dict("cityscapes"))
    bb, neck = m.backbone.to(DEV).train(), m.neck.to(DEV).train()
    x = images(2, 128, 256).to(DEV).half()
    gen = torch.Generator(device=DEV).manual_seed(4)
    gout = torch.randn(2, 256, 8, 16, device=DEV, generator=gen) * 1e-4
    params = [p for p in list(bb.parameters()) + list(neck.parameters()) if p.requires_grad]
    run = []
    try:
        for fold in (False, True):
            O.FOLD_READOUT_GRAD = fold
            for blk in bb.transformer.resblocks:
                blk.__dict__.pop("_dclip_dscale", None)  # fresh delayed-scale states per arm
            for _ in range(2):
                for p in params:
                    p.grad = None
                out = neck(bb(x))[0]
                (out.float() * gout).sum().backward()
            run.append([p.grad.clone() for p in params if p.grad is not None])
    finally:
        O.FOLD_READOUT_GRAD = True
    assert len(run[0]) == len(run[1]) >= 12 * 12
    worst = max(rel_err(b.float(), a.float()) for a, b in zip(*run))
    assert worst < 5e-3, worst


def test_fp16_delayed_scale_steps_match_exact():
    """ViT-B/16 fp16 backward, three passes with the same data: the first takes the exact scales
    and primes every block's DelayedScale; the later ones cast on the delayed scales (no
    grad_scale pass left in the blocks) and give the same gradients as the exact-scale path
    within fp16 rounding: identical data, so the delayed scale IS the exact one, but the
    delayed-scale LN backward contracts its row formula differently (ulps of fp32, which flip
    some fp16 roundings downstream).  The two exact passes agree to the order of the LN /
    bias-gradient atomics."""
    from denseclip_vit_multimodal_amd import ops
    m = _model(torch.float16)
    bb = m.backbone.train()
    x = images(1, 128, 256).to(DEV).half()
    gen = torch.Generator().manual_seed(7)
    ws = None
    grads = []
    for it in range(3):
        if it == 2:
            ops.FP16_DELAYED_SCALE = False  # exact scales again, as a reference
        try:
            bb.zero_grad(set_to_none=True)
            maps = bb(x)
            if ws is None:
                ws = [(torch.randn(mp.shape, generator=gen) * 1e-6).to(DEV) for mp in maps]
            sum((mp.float() * w).sum() for mp, w in zip(maps, ws)).backward()
            grads.append({n: p.grad.clone() for n, p in bb.named_parameters() if p.grad is not None})
        finally:
            ops.FP16_DELAYED_SCALE = True
    blk = bb.transformer.resblocks[3]
    assert blk.__dict__["_dclip_dscale"].primed == [True, True]
    worst = 0.0
    for n in grads[0]:
        assert rel_err(grads[0][n], grads[2][n]) < 1e-5, n
        e = rel_err(grads[1][n], grads[2][n])
        worst = max(worst, e)
        assert e < 3e-3, (n, e)  # fp16 rounding flips only (the fp16 model tests hold 3e-3)
    print("delayed vs exact scales, worst gradient rel. err.", worst)


def test_fp16_delayed_scale_overflow_is_flagged_and_reprimed():
    """ADVICE r4 (the delayed scales' overflow contract, ops.FP16_DELAYED_SCALE): a gradient that
    grows 1e5x between two backwards (past the 4096x margin) overflows in the delayed-scale fp16
    casts — the parameter gradients of that backward are NON-FINITE (a plain loop would apply
    them, as with GradScaler's scaled gradients; never silently wrong finite values), and
    train.nonfinite_flag (what train_step / step_unless_nonfinite compute) flags it and re-primes
    every site: the next backward takes exact scales and matches the exact-scale path, and the one
    after is on delayed scales again, within fp16 rounding of it."""
    from denseclip_vit_multimodal_amd import ops, train
    m = _model(torch.float16)
    bb = m.backbone.train()
    x = images(1, 128, 256).to(DEV).half()
    gen = torch.Generator().manual_seed(8)
    params = [p for p in bb.parameters() if p.requires_grad]
    opt = torch.optim.SGD(params, lr=0.0)  # only the parameter list nonfinite_flag checks
    ws = None

    def backward(c):
        nonlocal ws
        bb.zero_grad(set_to_none=True)
        maps = bb(x)
        if ws is None:
            ws = [(torch.randn(mp.shape, generator=gen) * 1e-6).to(DEV) for mp in maps]
        sum((mp.float() * (w * c)).sum() for mp, w in zip(maps, ws)).backward()
        return {n: p.grad.clone() for n, p in bb.named_parameters() if p.grad is not None}

    backward(1.0)  # exact scales; primes every site
    g2 = backward(1e5)
    assert not all(torch.isfinite(t).all() for t in g2.values())
    n0 = ops.STATS.get("fp16_scale_reprime", 0)
    flag = train.nonfinite_flag(opt, torch.zeros((), device=DEV))
    assert float(flag) == 1.0
    g3 = backward(1e5)  # re-primed: exact scales
    assert ops.STATS.get("fp16_scale_reprime", 0) == n0 + 1
    assert float(train.nonfinite_flag(opt, torch.zeros((), device=DEV))) == 0.0
    g4 = backward(1e5)  # delayed scales again (from g3's maxima)
    ops.FP16_DELAYED_SCALE = False
    try:
        ref = backward(1e5)
    finally:
        ops.FP16_DELAYED_SCALE = True
    for n in ref:
        assert torch.isfinite(g3[n]).all() and torch.isfinite(g4[n]).all(), n
        assert rel_err(g3[n], ref[n]) < 1e-5, n
        assert rel_err(g4[n], ref[n]) < 3e-3, n


def test_fp16_block_backward_under_graph_capture_takes_exact_scales():
    """an fp16 block backward captured with torch.cuda.graph does not use the delayed
    scales (their use counter is host state a replay cannot advance): with the block's
    DelayedScale primed, the captured backward equals the exact-scale eager backward bit for bit on
    every replay, also after the gradient grew 1e5x (which would overflow a frozen delayed scale)."""
    from denseclip_vit_multimodal_amd import ops
    from test_gpu_torch_ops import _block
    blk = _block()
    B, N, H, C = 2, 257, 12, 768
    ds = ops.DelayedScale()
    meta = (B, N, H, torch.float16, False, None, None, ds)
    x = torch.randn(B * N, C, device=DEV).requires_grad_(True)
    gy = torch.randn(B * N, C, device=DEV) * 1e-6
    scale = torch.ones((), device=DEV)

    def step():
        y = ops.BlockFn.apply(x, meta, *blk.hip_params())
        y.backward(gy * scale)
        return y

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):  # primes both sites, warms the allocator and the weight casts
            x.grad = None
            blk.zero_grad(set_to_none=True)
            step()
    torch.cuda.current_stream().wait_stream(s)
    assert ds.primed == [True, True]
    refs = []
    ops.FP16_DELAYED_SCALE = False
    try:
        for c in (1.0, 1e5):
            scale.fill_(c)
            x.grad = None
            blk.zero_grad(set_to_none=True)
            step()
            refs.append((x.grad.clone(), {n: p.grad.clone() for n, p in blk.named_parameters() if p.grad is not None}))
    finally:
        ops.FP16_DELAYED_SCALE = True
    x.grad = None
    blk.zero_grad(set_to_none=True)
    scale.fill_(1.0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for c, (gx_ref, gw_ref) in zip((1.0, 1e5), refs):
        scale.fill_(c)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(x.grad, gx_ref), c
        for n, p in blk.named_parameters():
            if n in gw_ref:
                assert torch.equal(p.grad, gw_ref[n]), (c, n)


@pytest.mark.parametrize("M,N,K", [(200, 256, 128), (4100, 768, 768), (16392, 3072, 768)])
def test_scaled_ops_equal_host_alpha(M, N, K):
    """gemm / weight_grad / cast / tokens_bwd with the device scale == the host-float path (the
    three shapes take the 128x128, 256x256 grid and persistent + M-tail GEMM kernels)."""
    from denseclip_vit_multimodal_amd import ops
    torch.manual_seed(0)
    g = torch.randn(M, K, device=DEV) * 3e-8
    ws = ops.grad_scale(g, torch.float16)
    s = host_scale(g)
    a_dev = ops.cast(g, torch.float16, scale_t=ws)
    a_host = ops.cast(g, torch.float16, s)
    assert torch.equal(a_dev, a_host)
    assert a_dev.abs().amax().item() > 4.0  # scaled up out of the fp16 subnormal range
    B = torch.randn(N, K, device=DEV).half()
    assert torch.equal(ops.gemm(a_dev, B, out_dtype=torch.float32, scale=ws),
                       ops.gemm(a_dev, B, out_dtype=torch.float32, alpha=1.0 / s))
    x = torch.randn(M, N, device=DEV).half()
    dw_dev, db_dev = ops.weight_grad(a_dev, x, scale=ws)
    dw_host, db_host = ops.weight_grad(a_dev, x, alpha=1.0 / s)
    assert torch.equal(dw_dev, dw_host)
    assert rel_err(db_dev, db_host) < 1e-6  # column sums: atomics, order-dependent rounding
    ref = g.double().t() @ x.double()
    assert rel_err(dw_dev, ref) < 2e-3


def test_tokens_bwd_device_scale():
    from denseclip_vit_multimodal_amd import ops
    B, P, C = 2, 64, 768
    dx = torch.randn(B * (P + 1), C, device=DEV) * 1e-8
    ws = ops.grad_scale(dx, torch.float16)
    s = host_scale(dx)
    d_dev = ops.D().tokens_bwd(dx, torch.float16, 1.0, B, P, ws)
    d_host = ops.D().tokens_bwd(dx, torch.float16, s, B, P)
    for a, b in zip(d_dev, d_host):
        assert torch.equal(a, b)


def _model(cdt):
    from denseclip_vit_multimodal_amd import DenseCLIP
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **CITYSCAPES_CFG)
    m.load_state_dict(spec_state_dict("cityscapes"))
    m.backbone.compute_dtype = cdt
    return m.to(DEV)


def test_fp16_backbone_backward_makes_no_host_sync():
    """ViT-B/16 fwd+bwd in fp16 (the gradient-scaled path through all 12 BlockFn and the
    patch embedding) under torch's sync debug mode "error": any device->host read raises."""
    m = _model(torch.float16)
    bb = m.backbone.train()
    x = images(1, 128, 256).to(DEV).half()
    gen = torch.Generator().manual_seed(5)
    ws = None
    for it in range(2):  # the second pass runs with every cache / allocation warm
        maps = bb(x)
        if ws is None:
            ws = [(torch.randn(mp.shape, generator=gen) * 1e-6).to(DEV) for mp in maps]
        torch.cuda.synchronize()
        if it == 1:
            torch.cuda.set_sync_debug_mode("error")
        try:
            loss = sum((mp.float() * w).sum() for mp, w in zip(maps, ws))
            loss.backward()
        finally:
            torch.cuda.set_sync_debug_mode(0)
        torch.cuda.synchronize()
    for name, p in bb.named_parameters():
        if p.grad is not None:
            assert torch.isfinite(p.grad).all(), name
    w = bb.transformer.resblocks[0].attn.in_proj_weight.grad
    assert w is not None and w.abs().sum() > 0


# ---------------------------------------------------------------------------- stochastic depth
def test_row_scale_add_matches_torch():
    from denseclip_vit_multimodal_amd import ops
    rows, cols, ntok = 3 * 257, 768, 257
    x, y = torch.randn(rows, cols, device=DEV), torch.randn(rows, cols, device=DEV)
    s = torch.rand(ntok, device=DEV)
    sr = s.repeat(rows // ntok)[:, None]
    assert torch.equal(ops.row_scale_add(x, y, s), x + sr * y)
    assert torch.equal(ops.row_scale_add(None, y, s), sr * y)


@pytest.mark.parametrize("cdt,tol", [(torch.float16, 3e-3), (torch.bfloat16, 2e-2)])
def test_block_drop_path_matches_torch_reference(cdt, tol):
    """BlockFn with stochastic-depth masks vs the reference block computed in fp32 torch on the
    LND layout (models.py:291-294: x + drop_path(attn(ln_1(x))), then the MLP branch; the mask has
    one value per token position), forward and the gradients of every input."""
    from denseclip_vit_multimodal_amd import ops
    from denseclip_vit_multimodal_amd.models import ResidualAttentionBlock
    torch.manual_seed(0)
    B, Ntok, C, H = 2, 257, 768, 12
    blk = ResidualAttentionBlock(C, H).to(DEV)
    with torch.no_grad():
        for p in blk.parameters():
            if p.dim() == 1:
                p.normal_(0, 0.02)
        blk.ln_1.weight.add_(1.0)
        blk.ln_2.weight.add_(1.0)
    keep = 0.7
    m1 = torch.empty(Ntok, device=DEV).bernoulli_(keep).div_(keep)
    m2 = torch.empty(Ntok, device=DEV).bernoulli_(keep).div_(keep)
    assert 0 < int((m1 == 0).sum()) < Ntok
    x = torch.randn(B, Ntok, C, device=DEV)
    w = torch.randn(B, Ntok, C, device=DEV)

    xr = x.clone().requires_grad_(True)
    xl = xr.transpose(0, 1)
    y = xl + m1[:, None, None] * blk.attention(blk.ln_1(xl))
    y = y + m2[:, None, None] * blk.mlp(blk.ln_2(y))
    ref = y.transpose(0, 1)
    (ref * w).sum().backward()
    gref = [xr.grad] + [p.grad.clone() for p in blk.hip_params()]
    blk.zero_grad(set_to_none=True)

    xh = x.reshape(B * Ntok, C).clone().requires_grad_(True)
    out = ops.BlockFn.apply(xh, (B, Ntok, H, cdt, False, None, (m1, m2)), *blk.hip_params())
    assert rel_err(out.view(B, Ntok, C), ref.detach()) < tol
    (out.view(B, Ntok, C) * w).sum().backward()
    got = [xh.grad.view(B, Ntok, C)] + [p.grad for p in blk.hip_params()]
    names = ["x", "ln1w", "ln1b", "w_in", "b_in", "w_out", "b_out", "ln2w", "ln2b", "w1", "b1", "w2", "b2"]
    for n, a, b in zip(names, got, gref):
        assert rel_err(a, b) < 3 * tol, (n, rel_err(a, b))


def test_vit_drop_path_training_step():
    """ViT-B/16 at drop_path_rate 0.2: eval is deterministic and equals the rate-0 model; a training
    forward draws fresh per-token masks (two draws differ) and its backward gives finite gradients."""
    from denseclip_vit_multimodal_amd.models import CLIPVisionTransformer
    torch.manual_seed(0)
    kw = dict(input_resolution=224, patch_size=16, width=768, layers=12, heads=12, out_indices=[3, 11],
              compute_dtype=torch.bfloat16)
    m = CLIPVisionTransformer(drop_path_rate=0.2, **kw).to(DEV)
    m0 = CLIPVisionTransformer(drop_path_rate=0.0, **kw).to(DEV)
    m0.load_state_dict(m.state_dict())
    x = images(1, 128, 256).to(DEV)
    with torch.no_grad():
        m.eval(), m0.eval()
        assert torch.equal(m(x)[-1], m0(x)[-1])
    m.train()
    a = m(x)
    with torch.no_grad():
        b = m(x)[-1]
    assert not torch.equal(a[-1].detach(), b)
    sum(t.float().sum() for t in a).backward()
    g = m.transformer.resblocks[11].mlp.c_fc.weight.grad
    assert g is not None and torch.isfinite(g).all() and g.abs().sum() > 0
