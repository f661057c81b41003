"""Torch-facing wrappers of the dclip custom ops and the autograd Functions of the ViT path.

Every op is a torch.ops.dclip.* custom op (TORCH_LIBRARY in csrc/torch_ops.cpp over the C ABI
of libdclip.so, fake implementations in _torch_ops.py) that launches one or more HIP kernels
on the current stream of the current device; tensors are only plumbing (device memory + the
caching allocator).  There is no CPU fallback: a CPU tensor or a missing library raises.

Numerics (the contract checked by tests/test_gpu_parity.py):
  * the residual stream, LayerNorm statistics, bias/LN gradients and weight gradients are
    fp32; GEMM/attention operands are the compute dtype (bf16 or fp16) with fp32 MFMA
    accumulation; softmax statistics are fp32.
"""
import math
import weakref

import torch

from . import _native as N

N_ = N

_DT = {torch.float32: N.F32, torch.float16: N.F16, torch.bfloat16: N.BF16}


def _dt(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}") from None


def _p(t):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


# Optional per-op device timing: set TIMING = {} to collect name -> [(start, end)] HIP
# events recorded on the launching stream around each op (bench.py uses it to derive the
# per-launch kernel duration inside its timed region).
TIMING = None
TIMING_OPS = False  # with TIMING: also every torch.ops.dclip launch, as "op:<name>" (bench's breakdown)
STATS = {}  # path counters (tests check which path ran)


def _stat(name):
    STATS[name] = STATS.get(name, 0) + 1


def _tic():
    if TIMING is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _toc(name, e0):
    if e0 is None:
        return
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record()
    TIMING.setdefault(name, []).append((e0, e1))


def timing_summary():
    """name -> (launches, total ms, mean ms); synchronises."""
    torch.cuda.synchronize()
    out = {}
    for k, evs in (TIMING or {}).items():
        tot = sum(a.elapsed_time(b) for a, b in evs)
        out[k] = (len(evs), tot, tot / max(1, len(evs)))
    return out


def _check(*ts, strided=()):
    """Every tensor on the GPU; contiguous unless listed in `strided` (ops that take explicit
    strides, e.g. channels-last pixel-row views)."""
    for t in ts + tuple(strided):
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("denseclip HIP op got a CPU tensor: the MI355X path has no CPU fallback")
    for t in ts:
        if t is not None and not t.is_contiguous():
            raise RuntimeError("denseclip HIP op needs contiguous tensors")


# ============================================================================ raw ops
# Each wrapper calls one torch.ops.dclip.* custom op (csrc/torch_ops.cpp, TORCH_LIBRARY over
# the C ABI of include/dclip.h): outputs come from the caching allocator, the kernels run on
# the current HIP stream.
_D = None


class _TimedOps:
    """torch.ops.dclip with HIP events around each launch (TIMING_OPS)."""

    def __init__(self, d):
        self._d = d

    def __getattr__(self, name):
        fn = getattr(self._d, name)

        def call(*a, **k):
            e0 = _tic()
            r = fn(*a, **k)
            _toc("op:" + name, e0)
            return r
        return call


def D():
    """torch.ops.dclip (loads libdclip_torch.so on first use; raises if it is missing)."""
    global _D
    if _D is None:
        from . import _torch_ops
        _D = _torch_ops.load()
    if TIMING_OPS and TIMING is not None:
        return _TimedOps(_D)
    return _D


def _env_option(opt, default=0):
    import os
    for kv in filter(None, os.environ.get("DCLIP_OPTIONS", "").split(",")):
        k, v = kv.split("=")
        if int(k) == opt:
            return int(v)
    return default


_GEMM_WALK = [_env_option(N.OPT_GEMM_SCHED)]  # the DCLIP_OPT_GEMM_SCHED value in force (DCLIP_OPTIONS at load)


def set_gemm_walk(walk):
    """Select the persistent NT GEMMs' tile walk for the launches that follow (DCLIP_OPT_GEMM_SCHED:
    0 static XCD-contiguous ranges, 1 every tile claimed — work-conserving when other kernels hold
    CUs, e.g. RCCL's channel kernels during a bucket all-reduce); returns the previous value.  The
    outputs are bitwise equal under either walk (test_gemm_work_conserving_walk_matches_static)."""
    prev = _GEMM_WALK[0]
    if walk != prev:
        N.call("dclip_set_option", N.OPT_GEMM_SCHED, int(walk))
        _GEMM_WALK[0] = int(walk)
    return prev


def layernorm_fwd(x2d, w, b, out_dtype, eps=1e-5):
    """(y in out_dtype, mean, rstd) of LayerNorm over the last dim in fp32 (models.py:243-249)."""
    _check(x2d, w, b)
    return D().layernorm_fwd(x2d, w, b, out_dtype, float(eps))


def layernorm_bwd(dy, x, w, mean, rstd, dw, db, res=None, lp_dtype=None, dy_scale=None, dy_ntok=0):
    """dx = res + LN^T(dy) (fp32; res optional); dw / db (fp32, zeroed by the caller) are
    accumulated in place.  With lp_dtype also returns lp = (lp_dtype) dx, the next GEMM's operand.
    dy_scale: a grad_scale() / HeadScale (s, 1/s, ..) buffer, dy read as dy * 1/s (an fp16 dy left on
    its gradient scale); dy_ntok > 0: dy's rows with row % dy_ntok == 0 (CLS) read as 0 (no lp)."""
    _check(dy, x, w, mean, rstd, dw, db, res, dy_scale)
    if lp_dtype is None:
        return D().layernorm_bwd(dy, x, w, mean, rstd, res, dw, db, dy_scale, int(dy_ntok))
    assert dy_ntok == 0
    return D().layernorm_bwd_lp(dy, x, w, mean, rstd, res, dw, db, lp_dtype, dy_scale)


def layernorm_bwd_add(dy, x, w, mean, rstd, dw, db, res, add, ntok, lp_dtype):
    """layernorm_bwd with res, plus `add` (a bf16 token buffer whose CLS rows, row % ntok == 0,
    read as 0) before the lp cast: (dx, lp) — dclip_layernorm_bwd_add."""
    _check(dy, x, w, mean, rstd, dw, db, res, add)
    e0 = _tic()
    out = D().layernorm_bwd_add(dy, x, w, mean, rstd, res, add, ntok, dw, db, lp_dtype)
    _toc("layernorm_bwd_add", e0)
    return out


# A bf16 read-out map's gradient folded into the NEXT block's ln_1 backward (which runs before
# the map's own block backward): dclip_layernorm_bwd_add writes the map's block-output gradient
# and its bf16 copy in one pass, and the map's block skips its dclip_add_readout_cast pass.
FOLD_READOUT_GRAD = True


class ReadoutLink:
    """Hand-over of one read-out map's gradient between two BlockFn backwards (FOLD_READOUT_GRAD).

    The producer of the map's gradient (NeckLevelsFn's backward, which runs before every block
    backward) stores it in `g`; the next block's backward adds it inside its ln_1 backward and
    stores the bf16 operand it wrote in `lp`; the map's own block then takes `lp` as its first
    GEMM operand when the gradient autograd hands it IS `g` (the map had no other consumer), and
    otherwise adds the difference.  Both fields are cleared by the map's block.

    fp16 (delayed scales): `ds` / `hsb` are the map block's DelayedScale and HeadScale buffer; the
    next block's ln_1 backward then adds the map gradient times the heads' 1/s and casts on the
    map block's MLP-site delayed scale (dclip_layernorm_bwd_scaled_add), handing over the scale
    pair in `pair` — only once that site is primed."""
    __slots__ = ("gh", "gw", "g", "lp", "ds", "hsb", "pair")

    def __init__(self, gh, gw, ds=None, hsb=None):
        self.gh, self.gw, self.ds, self.hsb = gh, gw, ds, hsb
        self.g = self.lp = self.pair = None


def gemm(A, B, epi=N.EPI_STORE, bias=None, aux=None, out_dtype=None, alpha=1.0, scale=None, lp_copy=False):
    """out[m][n] = alpha * sum_k A[m][k] B[n][k] (+ epilogue).  A: (M, K), B: (N, K).
    EPI_GELU returns (z, quick_gelu(z)).  scale: a grad_scale() buffer whose 1/s also
    multiplies the result (read on the device).  lp_copy (EPI_RESIDUAL only): returns (out, a
    copy of out in A's dtype) written by the same epilogue."""
    _check(A, B, bias, aux, scale)
    assert A.shape[1] == B.shape[1], (A.shape, B.shape)
    e0 = _tic()
    if lp_copy:
        assert epi == N.EPI_RESIDUAL and alpha == 1.0 and scale is None and out_dtype in (None, torch.float32)
        out = D().gemm_residual_lp(A, B, bias, aux)
    elif epi == N.EPI_GELU:
        out = D().gemm_gelu(A, B, bias)
    else:
        odt = out_dtype or (torch.float32 if epi == N.EPI_RESIDUAL else A.dtype)
        out = D().gemm(A, B, epi, bias, aux, odt, float(alpha), scale)
    _toc("gemm", e0)
    return out


def gemm_gelu_h(A, B, bias=None):
    """quick_gelu(A B^T + bias) alone: EPI_GELU without its pre-activation output (the forward of a
    block no backward will run through)."""
    _check(A, B, bias)
    e0 = _tic()
    out = D().gemm_gelu_h(A, B, bias)
    _toc("gemm", e0)
    return out


def transpose2d(x, out_dtype):
    """(rows, cols) -> (cols, rows) in out_dtype."""
    _check(x)
    return D().transpose2d(x, out_dtype)


def cast(x, dtype, scale=1.0, scale_t=None):
    """(dtype)(x * scale), times s of the grad_scale() buffer scale_t when given."""
    _check(x, scale_t)
    if x.dtype == dtype and scale == 1.0 and scale_t is None:
        return x
    return D().cast(x, dtype, float(scale), scale_t)


FP16_GRAD_AMAX = 16.0


def grad_scale(g, cdt):
    """Power-of-two scale for casting the fp32 gradient g to the compute dtype, ON THE DEVICE.

    bf16 has the fp32 exponent range: None (no scaling).  fp16 does not: the gradients of a
    segmentation loss averaged over ~10^5-10^7 pixels sit at 1e-5..1e-9, in (or below) fp16's
    subnormal range, so they are scaled by s = 2^floor(log2(FP16_GRAD_AMAX / max|g|)) before
    the cast and every fp32 result computed from them is unscaled by 1/s in the GEMM epilogue.
    Returns the (s, 1/s, 0, 0) f32 buffer dclip_grad_scale writes; cast / tokens_bwd read s from
    it and gemm / weight_grad read 1/s, all on the stream: no device->host round trip."""
    if cdt != torch.float16:
        return None
    g = g.detach()
    _check(g)
    return D().grad_scale(g if g.is_contiguous() else g.contiguous(), FP16_GRAD_AMAX)


# fp16 backward: the block gradients' casts on DELAYED scales (the previous step's maximum at the
# same site; dclip_add_readout_cast_scaled / dclip_layernorm_bwd_scaled) — one pass where the
# exact scale needs a maximum pass and a cast pass.  False: exact scales every step.
#
# Overflow contract (torch.cuda.amp.GradScaler's): a gradient that grows more than
# 65504 / FP16_GRAD_AMAX = 4096x between two backwards of a site overflows to inf in its
# fp16 copy, so that backward's parameter gradients are non-finite — never silently wrong finite
# values.  Such a step must be skipped: train.train_step / train.step_unless_nonfinite do it (a
# plain `loss.backward(); opt.step()` loop would apply the inf / NaN update, as it would with
# GradScaler's scaled gradients), and the non-finite flag they compute re-primes every site
# (watch_fp16_overflow), so the next backward takes exact scales and the one after is delayed
# again.  A backward captured into a graph (torch.cuda.graph) takes exact scales: the delayed
# scales' use counter is host state a replay could not advance.
FP16_DELAYED_SCALE = True


DS_STATE_FLOATS = 196  # DCLIP_DS_STATE_FLOATS (include/dclip.h)


_DELAYED = weakref.WeakSet()  # every DelayedScale (re-primed together after an overflowed step)
_OVERFLOW_WATCH = []  # (event, pinned host copy of a non-finite flag) not yet read


def watch_fp16_overflow(flag):
    """Queue a device-side non-finite-gradient flag (train.nonfinite_flag) for the delayed fp16
    scales: once the copy has landed (an event query, never a wait) a non-zero flag re-primes every
    site, so the next backward takes exact scales instead of scales from an overflowed step's
    maxima (whose non-finite values keep the previous, too large, scale at every later site)."""
    if not FP16_DELAYED_SCALE or not _DELAYED or not flag.is_cuda or torch.cuda.is_current_stream_capturing():
        return  # (the queue is drained only by delayed-scale backwards: nothing to queue without them)
    host = torch.empty((), dtype=torch.float32, pin_memory=True)
    host.copy_(flag.detach().reshape(()).float(), non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    _OVERFLOW_WATCH.append((ev, host))


def _poll_fp16_overflow():
    while _OVERFLOW_WATCH and _OVERFLOW_WATCH[0][0].query():
        _, host = _OVERFLOW_WATCH.pop(0)
        if float(host) != 0.0:
            _stat("fp16_scale_reprime")
            for ds in list(_DELAYED):
                ds.uses = [0, 0]


class DelayedScale:
    """Per-block state of the fp16 backward's delayed gradient scales, kept on the block module
    across training steps: site 0 = the MLP branch's incoming gradient, site 1 = the attention
    branch's.  A site's first backward takes the exact two-pass scale and seeds the state
    (`prime`); later ones cast with the scale of the previous backward's maximum at that site and
    record their own (include/dclip.h, dclip_add_readout_cast_scaled).  `uses[i]` counts the
    site's delayed calls (1, 2, ...: the kernels' `use`)."""

    def __init__(self):
        self.buf = None
        self.uses = [0, 0]
        _DELAYED.add(self)

    @property
    def primed(self):
        return [u > 0 for u in self.uses]

    def site(self, i, device):
        if self.buf is None or self.buf.device != device:
            self.buf = torch.zeros(2, DS_STATE_FLOATS, dtype=torch.float32, device=device)
            self.uses = [0, 0]
        return self.buf[i]

    def next_use(self, i):
        u = self.uses[i]
        self.uses[i] = u + 1
        return u

    def prime(self, i, pair):
        """Seed site i from the exact (s, 1/s, ..) pair of this backward: call 1 then reads a
        maximum of target / s, i.e. the scale s again (dclip.h's seeding rule)."""
        st = self.site(i, pair.device)
        st.zero_()
        st[0:1].copy_(FP16_GRAD_AMAX / pair[0:1])
        st[192:193].copy_(pair[0:1])
        self.uses[i] = 1


def add_readout_cast_scaled(a, b, ntok, b_scale, ds, i):
    """(a + b * 1/s_heads with b's CLS rows masked, or a when b is None; its fp16 copy on site i's
    delayed scale; the (s, 1/s) pair of that copy)."""
    st = ds.site(i, a.device)
    _check(a, b_scale, st, strided=(b,) if b is not None else ())
    sm, lp, pair = D().add_readout_cast_scaled(a, b, ntok, b_scale, st, ds.next_use(i), FP16_GRAD_AMAX)
    return (sm if b is not None else a), lp, pair


def layernorm_bwd_scaled(dy, x, w, mean, rstd, dw, db, res, ds, i, dy_scale=None):
    """layernorm_bwd with res and an fp16 copy of dx on site i's delayed scale: (dx, lp, pair).
    dy: fp32, or fp16 on the scale whose (s, 1/s) buffer is dy_scale."""
    st = ds.site(i, x.device)
    _check(dy, x, w, mean, rstd, dw, db, res, st, dy_scale)
    return D().layernorm_bwd_scaled(dy, x, w, mean, rstd, res, dw, db, st, ds.next_use(i), FP16_GRAD_AMAX, dy_scale)


def layernorm_bwd_scaled_add(dy, x, w, mean, rstd, dw, db, res, add, ntok, add_scale, ds, i, dy_scale=None):
    """layernorm_bwd with res, plus `add` (16-bit, CLS rows read as 0) times *add_scale (optional),
    and an fp16 copy on site i's delayed scale of the state `ds`: (dx, lp, pair).  dy: fp32, or
    fp16 on the scale whose (s, 1/s) buffer is dy_scale."""
    st = ds.site(i, x.device)
    _check(dy, x, w, mean, rstd, dw, db, res, add, add_scale, st, dy_scale)
    e0 = _tic()
    out = D().layernorm_bwd_scaled_add(dy, x, w, mean, rstd, res, add, add_scale, ntok, dw, db, st, ds.next_use(i),
                                       FP16_GRAD_AMAX, dy_scale)
    _toc("layernorm_bwd_add", e0)
    return out


def weight_grad(dy, x, want_bias=True, alpha=1.0, db=None, scale=None):
    """dW = alpha dy^T x (N x K, fp32) and db += alpha colsum(dy) for dy (M, N), x (M, K)
    (compute dtype); scale: a grad_scale() buffer whose 1/s also multiplies both.

    One "TN" MFMA GEMM reading both operands in their natural token-major layout (the
    reduction runs over the rows), split over the M tokens with a deterministic slab
    combine; no transposed copies."""
    _check(dy, x, db, scale)
    if want_bias and db is None:  # db: a caller-zeroed (Nn,) f32 buffer, or allocated here
        db = torch.zeros(dy.shape[1], dtype=torch.float32, device=dy.device)
    elif not want_bias:
        db = None
    e0 = _tic()
    dW = D().weight_grad(dy, x, float(alpha), db, scale)
    _toc("gemm_wgrad", e0)
    return dW, db


def gemm_tn(A, B):
    """out[m][n] = sum_k A[k][m] B[k][n] (f32)."""
    _check(A, B)
    return D().gemm_tn(A, B)


LOG2E = 1.4426950408889634


def qkv_scale_vector(C, H, device):
    """Per-column epilogue scale of the in-projection: q columns x d^-0.5 log2(e)
    (the attention kernels take log2-domain queries), k and v columns x 1."""
    key = (C, H, str(device))
    v = _QSCALE.get(key)
    if v is None:
        v = torch.ones(3 * C, dtype=torch.float32, device=device)
        v[:C] = (C // H) ** -0.5 * LOG2E
        _QSCALE[key] = v
    return v


_QSCALE = {}


def attn_fwd(qkv, B, Ntok, H, scale):
    """qkv with the q columns pre-multiplied by scale*log2(e) (qkv_scale_vector)."""
    _check(qkv)
    e0 = _tic()
    o, lse = D().attn_fwd(qkv, B, Ntok, H, float(scale))
    _toc("attn_fwd", e0)
    return o, lse


def attn_fwd_fp8(qkv, B, Ntok, H):
    """fp8 (e4m3) attention forward (BASELINE config 5): the same qkv / o / lse contract as
    attn_fwd, on the block-scaled fp8 MFMA (dclip_attn_fwd_fp8)."""
    _check(qkv)
    e0 = _tic()
    o, lse = D().attn_fwd_fp8(qkv, B, Ntok, H)
    _toc("attn_fwd_fp8", e0)
    return o, lse


# configs[4]: True runs the backward of an fp8-forward block with its dK / dV pass on the block-scaled
# e4m3 MFMA too (dclip_attn_bwd_fp8).  Off by default: measured no faster than the 16-bit pass (dkdv8
# 2.88 vs dkdv6 2.84 ms per launch + a 50 us pack, profiles/r06/r6f) — that loop is issue-bound on the
# per-element softmax VALU, not on the MFMA cycles the e4m3 products save
ATTN_BWD_FP8 = False


def attn_bwd(qkv, o, dout, lse, B, Ntok, H, scale, fp8=False):
    _check(qkv, o, dout, lse)
    e0 = _tic()
    if fp8:
        dqkv = D().attn_bwd_fp8(qkv, o, dout, lse, B, Ntok, H, float(scale))
    else:
        dqkv = D().attn_bwd(qkv, o, dout, lse, B, Ntok, H, float(scale))
    _toc("attn_bwd", e0)
    return dqkv


def im2col(img, p, out_dtype):
    """Patch rows (B*gh*gw, K_pad): K = Cin*p*p zero-padded to a multiple of 64 (the GEMM's K
    step; p = 14 gives 588 -> 640)."""
    _check(img)
    return D().im2col(img, p, out_dtype)


def _patch_weight(conv_w, cdt, k_pad):
    """conv1 weight as GEMM rows (C, K_pad) in cdt, zero columns past Cin*p*p."""
    K = conv_w[0].numel()
    if K == k_pad:
        return WEIGHTS.get(conv_w, cdt)
    return WEIGHTS.get_with(conv_w, cdt, ("kpad", k_pad),
                            lambda w: torch.nn.functional.pad(w.reshape(w.shape[0], -1).float(), (0, k_pad - K)))


def pos_interp(pos, g, H, W):
    _check(pos)
    return D().pos_interp(pos, g, H, W)


def pos_interp_bwd(dout, g, H, W):
    _check(dout)
    return D().pos_interp_bwd(dout, g, H, W)


def row_scale_add(x, y, s):
    """(x or 0) + s[row % len(s)] * y for f32 (rows, C) token buffers: a residual branch under a
    per-token stochastic-depth mask (see BlockFn meta[6])."""
    _check(x, y, s)
    return D().row_scale_add(x, y, s)


def row_mean(x, B, rows, row_off=0, bstride=None):
    """(B, C) f32 mean over `rows` pixel rows per image of a row-major (.., C) tensor whose image b
    starts at row b*bstride/C + row_off (a ViT token buffer: bstride N*C, row_off 1)."""
    C = x.shape[-1]
    bstride = rows * C if bstride is None else bstride
    return D().row_mean(x, bstride, row_off, C, B, rows, C)


def score_map(v, text, B, HW, row_off=0, bstride=None, eps=1e-12):
    """v: pixel embedding rows (.., C) (image b's pixel p at row b*bstride/C + row_off + p);
    text (B, K, C) f32 -> (B, K, HW) f32."""
    text = text.float().contiguous()
    _check(text)
    C = v.shape[-1]
    bstride = HW * C if bstride is None else bstride
    return D().score_map(v, bstride, row_off, C, text, B, HW, float(eps))


def score_concat(tgt, score):
    """torch.cat([tgt, upsample(score, tgt's size).to(tgt.dtype)], dim=1) — the score_concat_index
    branch (denseclip.py:684-694) — as one HIP pass when tgt is a 16-bit read-out map over its token
    buffer (the backbone's maps): a channels-last (B, C + K, h, w) result, no resized score map or
    concatenation copy in HBM.  Other inputs take the resize + torch.cat it replaces."""
    score = score.contiguous()
    _check(score)  # tgt is a strided view by design (token_rows below)
    B, C, h, w = tgt.shape
    tok = token_rows(tgt)
    if tok is None or tgt.dtype not in (torch.bfloat16, torch.float16) or score.dtype != torch.float32 \
            or score.dim() != 4 or score.shape[1] > 64:
        return torch.cat([tgt, upsample(score, (h, w)).to(tgt.dtype)], dim=1)
    out = D().score_concat(tok, (h * w + 1) * C, 1, C, C, score, B, h, w)
    return out.view(B, h, w, C + score.shape[1]).permute(0, 3, 1, 2)


def bilinear(x, Ho, Wo, out_dtype=torch.float32):
    _check(x)
    return D().bilinear(x, Ho, Wo, out_dtype)


def bilinear_bwd(dout, Hi, Wi):
    dout = dout.contiguous()
    _check(dout)
    return D().bilinear_bwd(dout, Hi, Wi)


# ============================================================================ weight cache
# Every optimizer step (any torch.optim optimizer, fused or not) stamps the parameters IT holds
# with a new step number.  The fused AdamW kernel updates parameters in place WITHOUT moving their
# version counters, so the version alone cannot tell a cached compute-dtype copy that its master
# weight changed; frozen parameters (mode R's backbone) keep their stamp and their cached copies.
_GENERATION = [0]   # bumped by invalidate_weight_cache(): every entry is stale
_STEP = [0]


def _stamp_stepped_params(opt, *_):
    _STEP[0] += 1
    for group in opt.param_groups:
        for p in group["params"]:
            p.__dict__["_dclip_step"] = _STEP[0]
    if EAGER_WEIGHT_REFRESH:
        refresh_weight_copies([p for group in opt.param_groups for p in group["params"]])


# rewrite the cached 16-bit copies of the stepped weights right after the step, all in one launch
# per (device, dtype) (misc.hip weight_refresh_kernel), instead of one cast / transpose launch per
# weight at its first use in the next forward / backward
EAGER_WEIGHT_REFRESH = True
# bf16 blocks: the dX GEMMs feeding the two LayerNorm backward passes write their gradient in bf16
# instead of fp32 — 100 MB less written by the GEMM and read by the LN pass per call at the
# headline shape.  An intentional precision trade-off of the bf16 THROUGHPUT line, not reference
# parity (the reference trains in fp32 and has no autocast): one more bf16 rounding of each LN
# input gradient, which tests/emulation16.py models and tests/test_gpu_grad_parity.py bounds
# against the fp32 reference restatement.
LN_DY_LP = True
# The fp16 counterpart (ABI 6): the dX GEMMs write fp16 on the gradient scale their operand carries
# (no 1/s in their epilogue) and the LN backward applies the 1/s on load (dy_scale) — the same
# 100 MB per call.  One fp16 rounding (2^-11 relative, on a scale that keeps the values out of the
# subnormals) of each LN input gradient: 8x finer than the bf16 line's, modelled by
# tests/emulation16.py and bounded by tests/test_gpu_grad_parity.py like it; the forward outputs the
# 1e-3 parity is stated on are untouched.  Overflow (a gradient growing > 4096x between the operand's
# scale and the dX output) follows FP16_DELAYED_SCALE's contract: inf, flagged, the step skipped.
LN_DY_LP_FP16 = True
_REFRESH_DESC = {}  # (device, dtype) -> (key, device descriptor, tiles, pinned host copy)


def refresh_weight_copies(params):
    """Refresh, in place, the plain and transposed compute-dtype copies WEIGHTS holds for these
    fp32 parameters (the entries earlier forwards / backwards created), and re-stamp them valid.
    The copies keep their storage, so the device descriptor of the launch is built once and
    reused while the set of copies is unchanged.  A no-op for parameters without cached copies;
    derived layouts (get_with) stay lazy.  During stream capture (a whole train step captured into
    a graph, train.CapturedTrainStep) the launch is captured with the descriptor an eager step
    built, so every replay refreshes the copies after its optimizer step."""
    if not torch.cuda.is_available():
        return
    capturing = torch.cuda.is_current_stream_capturing()
    groups = {}
    for p in params:
        cache = p.__dict__.get("_dclip_cache")
        if not cache:
            continue
        w = p.detach()
        if not w.is_cuda or w.dtype != torch.float32 or not w.is_contiguous() or w.data_ptr() % 16:
            continue
        stamp = _Cast.stamp(p)
        rows = w.shape[0] if w.dim() else 1
        cols = w.numel() // max(rows, 1)
        for dt in (torch.bfloat16, torch.float16):
            ep, et = cache.get((dt, False)), cache.get((dt, True))
            vp = ep[1] if ep is not None else None
            vt = et[1] if et is not None else None
            if vp is not None and (vp.shape != (rows, cols) or vp.dtype != dt or not vp.is_contiguous()
                                   or vp.data_ptr() % 16 or vp.data_ptr() == w.data_ptr()):
                vp = None
            if vt is not None and (vt.shape != (cols, rows) or vt.dtype != dt or not vt.is_contiguous()
                                   or vt.data_ptr() % 16):
                vt = None
            if vp is None and vt is None:
                continue
            groups.setdefault((w.device, dt), []).append((cache, dt, w, vp, vt, stamp, rows, cols))
    for (dev, dt), items in groups.items():
        key = tuple((w.data_ptr(), 0 if vp is None else vp.data_ptr(), 0 if vt is None else vt.data_ptr(), r, c)
                    for _, _, w, vp, vt, _, r, c in items)
        ent = _REFRESH_DESC.get((dev, dt))
        if capturing and (ent is None or ent[0] != key):
            # a new descriptor needs a host -> device copy; replays without the refresh would read
            # stale copies: the set of copies must be the one an eager step already refreshed
            raise RuntimeError("refresh_weight_copies: the cached weight copies changed since the last eager "
                               "optimizer step; run one eager step before capturing the train step")
        if ent is None or ent[0] != key:
            table, tiles = [], 0
            for src, dp, dtp, r, c in key:
                tc = (c + 63) // 64
                table.append([src, dp, dtp, r, c, tiles, tc, 0])
                tiles += ((r + 63) // 64) * tc
            host = torch.tensor(table, dtype=torch.int64).pin_memory()
            desc = host.to(dev, non_blocking=True)
            ent = _REFRESH_DESC[(dev, dt)] = (key, desc, tiles, host)
        D().weight_refresh(ent[1], ent[2], dt)
        for cache, dt_, w, vp, vt, stamp, _, _ in items:
            if vp is not None:
                cache[(dt_, False)] = (stamp, vp)
            if vt is not None:
                cache[(dt_, True)] = (stamp, vt)


from torch.optim.optimizer import register_optimizer_step_post_hook  # noqa: E402

register_optimizer_step_post_hook(_stamp_stepped_params)


def invalidate_weight_cache():
    """Force every cached compute-dtype weight copy to be rebuilt on next use (for code that
    writes parameters through `.data` or outside torch.optim)."""
    _GENERATION[0] += 1


class _Cast:
    """Cache of the compute-dtype copy (and derived layouts) of fp32 master weights.

    The entries live ON the parameter object (attribute `_dclip_cache`), so they die with it:
    no entry outlives its parameter and no new parameter can inherit another's entry through
    a recycled `id`.  An entry is valid while the parameter's version counter, storage
    address, the last optimizer step that held it and the global generation are all unchanged."""

    @staticmethod
    def stamp(p):
        w = p.detach()
        return (_GENERATION[0], p.__dict__.get("_dclip_step", 0), w._version, w.data_ptr())

    @staticmethod
    def _lookup(p, key):
        w = p.detach()
        stamp = _Cast.stamp(p)
        cache = p.__dict__.get("_dclip_cache")
        if cache is None:
            cache = p.__dict__["_dclip_cache"] = {}
        ent = cache.get(key)
        if ent is not None and ent[0] == stamp:
            return w, cache, stamp, ent[1]
        return w, cache, stamp, None

    def get(self, p, dtype, transposed=False):
        w, cache, stamp, v = self._lookup(p, (dtype, transposed))
        if v is not None:
            return v
        w2 = w.reshape(w.shape[0], -1)
        if transposed:
            v = transpose2d(w2.contiguous(), dtype)
        else:
            v = cast(w2.contiguous(), dtype)
        cache[(dtype, transposed)] = (stamp, v)
        return v

    def get_with(self, p, dtype, tag, fn):
        """Cached fn(p) (a derived layout of parameter p in dtype), refreshed when p changes."""
        w, cache, stamp, v = self._lookup(p, (dtype, tag))
        if v is not None:
            return v
        v = fn(w).to(dtype).contiguous()
        cache[(dtype, tag)] = (stamp, v)
        return v


WEIGHTS = _Cast()


# ============================================================================ autograd
class PatchEmbedFn(torch.autograd.Function):
    """conv1 (patchify GEMM) + CLS + interpolated pos-embed + ln_pre
    (reference models.py:543-559).  Returns the fp32 residual stream (B*N, C)."""

    @staticmethod
    def forward(ctx, img, conv_w, cls, pos, ln_w, ln_b, patch, cdt):
        B, _, Hin, Win = img.shape
        C = conv_w.shape[0]
        gh, gw = Hin // patch, Win // patch
        P = gh * gw
        g = int(math.isqrt(pos.shape[0] - 1))
        # models.py:518: the embedding is used as-is whenever the token COUNT matches
        interp = (P != pos.shape[0] - 1)
        posf = pos_interp(pos.detach().contiguous(), g, gh, gw) if interp else pos.detach().contiguous()
        patches = im2col(img.contiguous(), patch, cdt)
        emb = gemm(patches, _patch_weight(conv_w, cdt, patches.shape[1]), out_dtype=torch.float32)
        x_pre = D().tokens_fwd(emb, cls.detach().float().contiguous(), posf, B, P)
        x, mean, rstd = layernorm_fwd(x_pre, ln_w.detach(), ln_b.detach(), torch.float32)
        ctx.save_for_backward(patches, x_pre, mean, rstd, ln_w)
        ctx.meta = (B, P, C, g, gh, gw, interp, cdt, tuple(conv_w.shape))
        return x

    @staticmethod
    def backward(ctx, dx):
        patches, x_pre, mean, rstd, ln_w = ctx.saved_tensors
        B, P, C, g, gh, gw, interp, cdt, wshape = ctx.meta
        dx = dx.contiguous()
        need = ctx.needs_input_grad
        dlnw = torch.zeros(C, dtype=torch.float32, device=dx.device)
        dlnb = torch.zeros(C, dtype=torch.float32, device=dx.device)
        dxp = layernorm_bwd(dx, x_pre, ln_w.detach(), mean, rstd, dlnw, dlnb)
        s = grad_scale(dxp, cdt) if need[1] else None
        demb, dcls, dposf = D().tokens_bwd(dxp, cdt, 1.0, B, P, s)
        dpos = None
        if need[3]:
            dpos = pos_interp_bwd(dposf, g, gh, gw) if interp else dposf
        dconv = None
        if need[1]:
            dW, _ = weight_grad(demb, patches, want_bias=False, scale=s)
            K = math.prod(wshape[1:])
            dconv = (dW if dW.shape[1] == K else dW[:, :K]).reshape(wshape)
        return (None, dconv, dcls if need[2] else None, dpos, dlnw if need[4] else None,
                dlnb if need[5] else None, None, None)


class BlockFn(torch.autograd.Function):
    """One ResidualAttentionBlock on the fp32 residual stream (reference models.py:291-294):
        x = x + out_proj(attn(qkv(ln_1(x))))
        x = x + c_proj(quick_gelu(c_fc(ln_2(x))))
    LN -> GEMM(+bias) -> fused attention -> GEMM(+bias+residual) -> LN -> GEMM(+bias+QuickGELU)
    -> GEMM(+bias+residual): 7 kernels, no elementwise passes.

    meta[5] (optional, may be None) = (gh, gw, map dtype): the block also returns the per-layer
    read-out map of its output (models.py:577-597 without ln_post; the layout of ReadoutFn), so the
    backward receives the map's gradient beside the residual one and folds it into the cast that
    feeds its first GEMM (dclip_add_readout_cast) instead of autograd summing two fp32 token
    gradients.

    meta[6] (optional) = (m1, m2): stochastic depth in training (reference models.py:257-268,
    291-294): f32 (Ntok,) keep masks already divided by the keep probability, one value per token
    POSITION (timm's drop_path on the reference's LND layout); the attention / MLP branch is
    added as x + m[token] * branch (dclip_row_scale_add) instead of through the fused residual
    epilogue, and its gradient is scaled the same way.

    meta[8] / meta[9] (optional, bf16 only) = the previous block's / this block's ReadoutLink
    (FOLD_READOUT_GRAD): the previous block's map gradient is added inside this block's ln_1
    backward (dclip_layernorm_bwd_add), and this block's own map gradient arrives already added
    to dxo, with its bf16 operand, from the next block's."""

    @staticmethod
    def forward(ctx, x, meta, ln1w, ln1b, w_in, b_in, w_out, b_out, ln2w, ln2b, w1, b1, w2, b2):
        B, Ntok, H, cdt, fp8 = meta[:5]
        ro = meta[5] if len(meta) > 5 else None
        dp = meta[6] if len(meta) > 6 else None
        C = x.shape[1]
        scale = (C // H) ** -0.5
        xh1, mu1, rs1 = layernorm_fwd(x, ln1w.detach(), ln1b.detach(), cdt)
        qkv = gemm(xh1, WEIGHTS.get(w_in, cdt), N.EPI_STORE_SCALED, bias=b_in.detach(),
                   aux=qkv_scale_vector(C, H, x.device))
        o, lse = attn_fwd_fp8(qkv, B, Ntok, H) if fp8 else attn_fwd(qkv, B, Ntok, H, scale)
        if dp is None:
            xm = gemm(o, WEIGHTS.get(w_out, cdt), N.EPI_RESIDUAL, bias=b_out.detach(), aux=x)
        else:
            xm = row_scale_add(x, gemm(o, WEIGHTS.get(w_out, cdt), bias=b_out.detach(), out_dtype=torch.float32),
                               dp[0])
        xh2, mu2, rs2 = layernorm_fwd(xm, ln2w.detach(), ln2b.detach(), cdt)
        if any(ctx.needs_input_grad):
            z, h = gemm(xh2, WEIGHTS.get(w1, cdt), N.EPI_GELU, bias=b1.detach())
        else:  # no backward will run (frozen backbone, inference): h alone, z is never stored
            z, h = None, gemm_gelu_h(xh2, WEIGHTS.get(w1, cdt), b1.detach())
        lp = None
        if dp is None and ro is not None and ro[2] == cdt:
            # the read-out map's token buffer comes out of the residual epilogue itself
            xo, lp = gemm(h, WEIGHTS.get(w2, cdt), N.EPI_RESIDUAL, bias=b2.detach(), aux=xm, lp_copy=True)
        elif dp is None:
            xo = gemm(h, WEIGHTS.get(w2, cdt), N.EPI_RESIDUAL, bias=b2.detach(), aux=xm)
        else:
            xo = row_scale_add(xm, gemm(h, WEIGHTS.get(w2, cdt), bias=b2.detach(), out_dtype=torch.float32), dp[1])
        ctx.save_for_backward(x, mu1, rs1, xh1, qkv, o, lse, xm, mu2, rs2, xh2, z, h,
                              ln1w, w_in, w_out, ln2w, w1, w2)
        ctx.meta = meta
        if ro is None:
            return xo
        gh, gw, mdt = ro[:3]
        ctx.set_materialize_grads(False)  # an unused map (or block output) brings None, not zeros
        buf = lp if lp is not None else (xo.clone() if mdt == torch.float32 else cast(xo, mdt))
        return xo, buf.as_strided((B, C, gh, gw), (Ntok * C, 1, gw * C, C), C)

    @staticmethod
    def backward(ctx, dxo, dmap=None):
        (x, mu1, rs1, xh1, qkv, o, lse, xm, mu2, rs2, xh2, z, h,
         ln1w, w_in, w_out, ln2w, w1, w2) = ctx.saved_tensors
        # fp8 forward (BASELINE config 5): the backward is the bf16 / fp16 flash backward, P
        # recomputed from the 16-bit q, k against the fp8 forward's own lse and delta taken from
        # its o — the straight-through gradient of the quantised forward
        B, Ntok, H, cdt, fp8 = ctx.meta[:5]
        dp = ctx.meta[6] if len(ctx.meta) > 6 else None
        # fp16 delayed scales (meta[7], a DelayedScale): only on the plain residual form
        C = x.shape[1]
        capturing = torch.cuda.is_current_stream_capturing()
        ds = ctx.meta[7] if (len(ctx.meta) > 7 and cdt == torch.float16 and dp is None and FP16_DELAYED_SCALE
                             and C in (512, 768, 1024) and not capturing) else None  # the widths dclip_layernorm_bwd_scaled takes
        if ds is not None:
            _poll_fp16_overflow()
        scale = (C // H) ** -0.5
        need = ctx.needs_input_grad
        wg = any(need[2:])
        # every zero-initialised small gradient of the block from ONE zeroed arena (one fill
        # launch instead of eight): LN weights / biases (4C), biases of c_proj (C), c_fc (4C),
        # out_proj (C), in_proj (3C)
        arena = torch.zeros(13 * C, dtype=torch.float32, device=x.device)
        dln1w, dln1b, dln2w, dln2b = (arena[i * C:(i + 1) * C] for i in range(4))
        zb2, zb1, zbo, zbi = arena[4 * C:5 * C], arena[5 * C:9 * C], arena[9 * C:10 * C], arena[10 * C:13 * C]
        dy = None
        s1 = None  # set here when the fold below also produced the fp16 scale of the MLP gradient
        if dxo is None:
            dxo = torch.zeros(B * Ntok, C, dtype=torch.float32, device=x.device)
        dxo = dxo.contiguous()
        lk = ctx.meta[9] if len(ctx.meta) > 9 else None  # this block's read-out map (ReadoutLink)
        if lk is not None:
            g, lp, pair = lk.g, lk.lp, lk.pair
            lk.g = lk.lp = lk.pair = None
            if lp is not None:  # the next block's ln_1 backward already added g into dxo
                if dmap is g:
                    dy, s1, dmap = lp, pair, None
                else:  # other consumers joined the map's gradient after g: add the difference
                    _stat("readout_fold_fixup")
                    d = _readout_grad_dense(g, B, Ntok, lk.gh, lk.gw, C).neg_()
                    if dmap is not None:
                        d += _readout_grad_dense(dmap, B, Ntok, lk.gh, lk.gw, C)
                    dxo, dmap = dxo + _unscale_(d, lk.hsb), None
        if ds is not None and ds.primed[0] and dy is None:
            base = hsb = None
            if dmap is not None:
                gh, gw = ctx.meta[5][:2]
                hsb = ctx.meta[5][3] if len(ctx.meta[5]) > 3 else None
                base = _readout_grad_buffer(dmap, B, Ntok, gh, gw, C)
            if dmap is None or base is not None:
                # one pass: (+ the map gradient) and the fp16 operand on the delayed scale
                dxo, dy, s1 = add_readout_cast_scaled(dxo, base, Ntok, hsb, ds, 0)
                dmap = None
        if dmap is not None:  # the read-out map's gradient joins the block output's
            gh, gw = ctx.meta[5][:2]
            hsb = ctx.meta[5][3] if len(ctx.meta[5]) > 3 else None  # HeadScale buffer (fp16 heads)
            base = _readout_grad_buffer(dmap, B, Ntok, gh, gw, C)
            if base is not None and cdt == torch.bfloat16 and dp is None and hsb is None:
                # one pass: dxo + map gradient (CLS rows masked) in fp32, and its bf16 copy
                dxo, dy = D().add_readout_cast(dxo, base, Ntok, cdt, 1.0)
            elif base is not None and cdt == torch.float16 and dp is None:
                # one pass: dxo + the unscaled map gradient (CLS rows masked) in fp32 and the
                # power-of-two fp16 scale of that sum (grad_scale's pair), read by the cast below
                dxo, s1 = D().add_readout_amax(dxo, base, Ntok, hsb, FP16_GRAD_AMAX)
            elif base is not None:
                dr = base.float() if base.dtype != torch.float32 else base.clone()
                dr.view(B, Ntok, C)[:, 0].zero_()
                dxo = dxo + _unscale_(dr, hsb)
            else:
                dxo = dxo + _unscale_(_readout_grad_dense(dmap, B, Ntok, gh, gw, C), hsb)

        # ---- MLP: xo = xm + h W2^T + b2,  h = qgelu(z),  z = xh2 W1^T + b1
        # (s1, s2: device-side power-of-two gradient scales, None unless fp16 — see grad_scale)
        dbr = dxo if dp is None else row_scale_add(None, dxo, dp[1])  # the MLP branch's gradient
        if s1 is None:
            s1 = grad_scale(dbr, cdt)
        if dy is None:
            dy = cast(dbr, cdt, scale_t=s1)
        if ds is not None and not ds.primed[0]:
            ds.prime(0, s1)
        del dbr
        dz = gemm(dy, WEIGHTS.get(w2, cdt, transposed=True), N.EPI_GELU_BWD, aux=z)
        dW2 = db2 = dW1 = db1 = None
        if wg:
            dW2, db2 = weight_grad(dy, h, db=zb2, scale=s1)
        dy_lp = LN_DY_LP and cdt == torch.bfloat16 and s1 is None  # bf16: no gradient scale
        # fp16: the dX GEMMs' outputs stay on their operand's gradient scale (no 1/s in the epilogue)
        # and go to the LN backward in fp16, which takes the 1/s on load (dy_scale; fast widths only)
        dy16 = LN_DY_LP_FP16 and cdt == torch.float16 and C in (512, 768, 1024)
        dxh2 = gemm(dz, WEIGHTS.get(w1, cdt, transposed=True), out_dtype=cdt if (dy_lp or dy16) else torch.float32,
                    scale=None if dy16 else s1)
        dsc1 = s1 if dy16 else None
        if wg:
            dW1, db1 = weight_grad(dz, xh2, db=zb1, scale=s1)
        del dz
        dyo = None
        if cdt == torch.bfloat16 and dp is None:  # no gradient scaling: the attention branch's operand comes out of the LN pass
            dxm, dyo = layernorm_bwd(dxh2, xm, ln2w.detach(), mu2, rs2, dln2w, dln2b, res=dxo, lp_dtype=cdt)
            s2 = None
        elif ds is not None and ds.primed[1]:  # fp16: the operand on the delayed scale, same pass
            dxm, dyo, s2 = layernorm_bwd_scaled(dxh2, xm, ln2w.detach(), mu2, rs2, dln2w, dln2b, dxo, ds, 1, dsc1)
        else:
            dxm = layernorm_bwd(dxh2, xm, ln2w.detach(), mu2, rs2, dln2w, dln2b, res=dxo, dy_scale=dsc1)
        del dxh2
        # ---- attention: xm = x + o Wout^T + bout
        if dyo is None:
            dab = dxm if dp is None else row_scale_add(None, dxm, dp[0])  # the attention branch's gradient
            s2 = grad_scale(dab, cdt)
            dyo = cast(dab, cdt, scale_t=s2)
            del dab
            if ds is not None:
                ds.prime(1, s2)
        do = gemm(dyo, WEIGHTS.get(w_out, cdt, transposed=True))
        dWo = dbo = dWi = dbi = None
        if wg:
            dWo, dbo = weight_grad(dyo, o, db=zbo, scale=s2)
        del dyo
        dqkv = attn_bwd(qkv, o, do, lse, B, Ntok, H, scale, fp8=bool(fp8) and ATTN_BWD_FP8)  # linear in dO: carries s2
        del do
        dxh1 = gemm(dqkv, WEIGHTS.get(w_in, cdt, transposed=True),
                    out_dtype=cdt if (dy_lp and s2 is None) or dy16 else torch.float32, scale=None if dy16 else s2)
        dsc2 = s2 if dy16 else None
        if wg:
            dWi, dbi = weight_grad(dqkv, xh1, db=zbi, scale=s2)
        del dqkv
        lk = ctx.meta[8] if len(ctx.meta) > 8 else None  # the previous block's read-out map
        base = None
        if lk is not None and lk.g is not None and need[0] and C in (512, 768, 1024):  # dclip_layernorm_bwd_add's widths
            base = _readout_grad_buffer(lk.g, B, Ntok, lk.gh, lk.gw, C)
            if lk.ds is None:
                base = base if base is not None and base.dtype == torch.bfloat16 else None
            elif capturing or not (lk.ds.primed[0] and dxh1.dtype in (torch.float32, torch.float16)
                                   and x.dtype == torch.float32):
                base = None
        if base is not None:
            _stat("readout_fold")
        if base is not None and lk.ds is None:  # its gradient and the previous block's first GEMM operand from this pass
            dxm, lk.lp = layernorm_bwd_add(dxh1, x, ln1w.detach(), mu1, rs1, dln1w, dln1b, dxm, base, Ntok,
                                           torch.bfloat16)
        elif base is not None:  # fp16: on the previous block's MLP-site delayed scale
            dxm, lk.lp, lk.pair = layernorm_bwd_scaled_add(dxh1, x, ln1w.detach(), mu1, rs1, dln1w, dln1b, dxm, base,
                                                           Ntok, lk.hsb, lk.ds, 0, dsc2)
        else:
            dxm = layernorm_bwd(dxh1, x, ln1w.detach(), mu1, rs1, dln1w, dln1b, res=dxm, dy_scale=dsc2)
        g = lambda i, t: t if need[i] else None  # noqa: E731
        return (dxm if need[0] else None, None, g(2, dln1w), g(3, dln1b), g(4, dWi), g(5, dbi), g(6, dWo),
                g(7, dbo), g(8, dln2w), g(9, dln2b), g(10, dW1), g(11, db1), g(12, dW2), g(13, db2))


def token_rows(m):
    """The (B*N, C) token buffer behind a read-out map (the channels-last view ReadoutFn /
    BlockFn return: strides (N*C, 1, W*C, C), offset C past the buffer start), or None."""
    if m.dim() != 4 or not m.is_cuda:
        return None
    B, C, gh, gw = m.shape
    Ntok = gh * gw + 1
    if m.stride() == (Ntok * C, 1, gw * C, C) and m.storage_offset() >= C and \
            m.untyped_storage().nbytes() >= (m.storage_offset() - C + B * Ntok * C) * m.element_size():
        return m.as_strided((B * Ntok, C), (C, 1), m.storage_offset() - C)
    return None


def _readout_grad_buffer(dmap, B, Ntok, gh, gw, C):
    """The read-out map's gradient as a (B*Ntok, C) token buffer whose CLS rows are NOT zeroed
    (callers mask them), when it already has the token-buffer layout (Conv3x3Fn's input
    gradient: zero copy); None otherwise."""
    if dmap.stride() == (Ntok * C, 1, gw * C, C) and dmap.storage_offset() >= C and \
            dmap.untyped_storage().nbytes() >= (dmap.storage_offset() - C + B * Ntok * C) * dmap.element_size():
        _stat("readout_zero_copy")
        return dmap.as_strided((B * Ntok, C), (C, 1), dmap.storage_offset() - C)
    return None


def _readout_grad_dense(dmap, B, Ntok, gh, gw, C):
    """The read-out map's gradient scattered into a fresh fp32 (B*Ntok, C) token gradient."""
    dy = torch.zeros(B * Ntok, C, dtype=torch.float32, device=dmap.device)
    dy.view(B, Ntok, C)[:, 1:].copy_(dmap.permute(0, 2, 3, 1).reshape(B, gh * gw, C))
    return dy


class ReadoutFn(torch.autograd.Function):
    """Per-layer dense read-out (reference models.py:568-582): optional ln_post (only for the
    last block, models.py:574-576), drop CLS, (B, N, C) -> (B, C, H, W).

    The map is returned as a channels-last VIEW of a token buffer (B*N, C) in the map dtype
    (strides (N*C, 1, W*C, C), offset C: the CLS row of each batch is skipped), so the neck's
    implicit-GEMM convs read the tokens in place: one cast (or the ln_post output) instead
    of an NCHW transpose.  `.contiguous()` gives the reference's NCHW layout."""

    @staticmethod
    def forward(ctx, x, ln_w, ln_b, meta):
        B, Ntok, gh, gw, out_dtype = meta[:5]
        C = x.shape[1]
        mean = rstd = None
        if ln_w is not None:
            buf, mean, rstd = layernorm_fwd(x, ln_w.detach(), ln_b.detach(), out_dtype)
        elif out_dtype == torch.float32:
            buf = x.clone()
        else:
            buf = cast(x, out_dtype)
        ctx.save_for_backward(x if ln_w is not None else None, mean, rstd, ln_w)
        ctx.meta = meta
        ctx.has_ln = ln_w is not None
        return buf.as_strided((B, C, gh, gw), (Ntok * C, 1, gw * C, C), C)

    @staticmethod
    def backward(ctx, dmap):
        x, mean, rstd, ln_w = ctx.saved_tensors
        B, Ntok, gh, gw, _ = ctx.meta[:5]
        hsb = ctx.meta[5] if len(ctx.meta) > 5 else None  # HeadScale buffer (fp16 heads)
        C = dmap.shape[1]
        base = _readout_grad_buffer(dmap, B, Ntok, gh, gw, C)
        if base is not None and ctx.has_ln and C in (512, 768, 1024):
            # ln_post's backward straight from the 16-bit token buffer: CLS rows masked and the heads'
            # 1/s applied on load (no fp32 copy, no in-place unscale pass)
            dw = torch.zeros(C, dtype=torch.float32, device=dmap.device)
            db = torch.zeros(C, dtype=torch.float32, device=dmap.device)
            dx = layernorm_bwd(base, x, ln_w.detach(), mean, rstd, dw, db, dy_scale=hsb, dy_ntok=Ntok)
            return dx, dw, db, None
        if base is not None:  # token-buffer layout (Conv3x3Fn's input gradient): take the buffer as it is
            dy = base.float() if base.dtype != torch.float32 else base.clone()
            dy.view(B, Ntok, C)[:, 0].zero_()
        else:
            dy = _readout_grad_dense(dmap, B, Ntok, gh, gw, C)
        _unscale_(dy, hsb)
        if not ctx.has_ln:
            return dy, None, None, None
        dw = torch.zeros(C, dtype=torch.float32, device=dy.device)
        db = torch.zeros(C, dtype=torch.float32, device=dy.device)
        dx = layernorm_bwd(dy, x, ln_w.detach(), mean, rstd, dw, db)
        return dx, dw, db, None


def bn_supported(x):
    """Train-mode BatchNorm on the HIP kernels: 16-bit channels-last maps, C % 8 == 0, C <= 2048."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float16)):
        return False
    C = x.shape[1]
    return C % 8 == 0 and 8 <= C <= 2048 and x.numel() > 0 and x.is_contiguous(memory_format=torch.channels_last)


class BatchNormFn(torch.autograd.Function):
    """nn.BatchNorm2d in train mode (batch statistics; the running statistics updated in place
    like torch's), optionally followed by the ReLU of a ConvModule / FCNHead (fused: the backward
    recomputes the mask from x), on a channels-last map viewed as (B*H*W, C): dclip_bn_fwd /
    dclip_bn_bwd (reference models.py:13-20 ConvModule norm + act, heads' FCNHead norm + ReLU)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, relu=False):
        w = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        _check(w, b, running_mean, running_var, strided=(x,))
        y, mean, rstd = D().bn_fwd(x, w, b, running_mean, running_var, float(momentum), float(eps), bool(relu))
        ctx.save_for_backward(x, w, b, mean, rstd)
        ctx.has_w = (weight is not None, bias is not None)
        ctx.relu = bool(relu)
        ctx.hsb = _head_scale_buf()
        _stat("bn_train")
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, mean, rstd = ctx.saved_tensors
        dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        # dw / db unscaled by the heads' 1/s inside the kernel (dx keeps the scale)
        dx, dw, db = D().bn_bwd(dy, x, w, b, mean, rstd, ctx.relu, ctx.has_w[0], ctx.has_w[1], ctx.hsb)
        return dx, (dw if ctx.has_w[0] else None), (db if ctx.has_w[1] else None), None, None, None, None, None


def bn_train(bn, x, relu=False):
    """`bn` (an nn.BatchNorm2d in train mode) on x via BatchNormFn, then the fused ReLU; the
    module's num_batches_tracked advances as torch's does.  Caller checks bn_supported(x)."""
    if bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    return BatchNormFn.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps, relu)


def bn_eval(bn, x, relu=False):
    """`bn` (an nn.BatchNorm2d in eval mode with running statistics) on x via dclip_bn_eval, with
    the following ReLU fused when relu.  No autograd (eval).  Caller checks bn_eval_ok."""
    w = bn.weight.detach() if bn.weight is not None else None
    b = bn.bias.detach() if bn.bias is not None else None
    _check(w, b, bn.running_mean, bn.running_var, strided=(x,))
    _stat("bn_eval")
    return D().bn_eval(x, w, b, bn.running_mean, bn.running_var, float(bn.eps), bool(relu))


def bn_eval_ok(bn, x):
    """Whether eval-mode `bn` runs on dclip_bn_eval for x (no gradient needed through it)."""
    f32 = all(t is None or t.dtype == torch.float32 for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var))
    needs_grad = torch.is_grad_enabled() and (x.requires_grad or any(
        p is not None and p.requires_grad for p in (bn.weight, bn.bias)))
    return (not bn.training and bn.track_running_stats and bn.running_mean is not None and f32
            and not needs_grad and bn_supported(x))


def bn_hip_ok(bn, x):
    """Whether `bn` in its current mode runs on the HIP batch-norm kernels for input x."""
    f32 = all(t is None or t.dtype == torch.float32 for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var))
    return bn.training and bn.track_running_stats and bn.momentum is not None and f32 and bn_supported(x)


class UpsampleFn(torch.autograd.Function):
    """F.interpolate(mode='bilinear', align_corners=False) to (Ho, Wo), fp32 output
    (reference denseclip.py:847, 860, 899, 909)."""

    @staticmethod
    def forward(ctx, x, Ho, Wo):
        ctx.shape = x.shape
        ctx.in_dtype = x.dtype
        return bilinear(x.contiguous(), Ho, Wo, torch.float32)

    @staticmethod
    def backward(ctx, dout):
        _, _, Hi, Wi = ctx.shape
        din = bilinear_bwd(dout, Hi, Wi)
        return din.to(ctx.in_dtype) if ctx.in_dtype != torch.float32 else din, None, None


def upsample(x, size):
    Ho, Wo = int(size[0]), int(size[1])
    return UpsampleFn.apply(x, Ho, Wo)


# ============================================================================ 16-bit neck / heads for fp32 images
class HeadScale:
    """Gradient scale of one forward's 16-bit neck / heads / read-out backward (fp32 images, the
    reference trainer's input, run through the HIP neck and heads in the backbone's compute dtype).

    The segmentation-loss gradients reaching the heads are ~1e-5..1e-8 per low-res logit: in or
    below fp16's subnormal range.  HeadsOutFn's backward therefore casts them to fp16 with a
    device-side power-of-two scale s (grad_scale; written into `buf` = (s, 1/s, 0, 0), no host
    sync) and every fp32 result computed from them downstream — the neck / head weight and BN
    gradients, the read-out maps' gradients entering the ViT backward — is multiplied by 1/s
    from `buf` by the op that produces it.  bf16 has the fp32 exponent range: no scaling.

    `torch_fallback` is set when any neck / head op ran on torch instead of a scale-aware HIP
    op with gradients on; HeadsOutFn then leaves s = 1 (the torch op's parameter gradients could
    not be unscaled)."""

    def __init__(self, device, cdt):
        self.cdt = cdt
        self.buf = None
        if cdt == torch.float16 and torch.is_grad_enabled():
            # built on the device (a host tensor would be a pageable copy + stream sync per forward)
            self.buf = torch.ones(4, dtype=torch.float32, device=device)
            self.buf[2:].zero_()
        self.torch_fallback = False


_HEAD_SCALE = [None]


class head_scale:
    """Context manager: the neck / head / read-out autograd Functions created inside it capture
    `hs.buf` and unscale their fp32 gradients by its 1/s."""

    def __init__(self, hs):
        self.hs = hs

    def __enter__(self):
        self.prev = _HEAD_SCALE[0]
        _HEAD_SCALE[0] = self.hs
        return self.hs

    def __exit__(self, *exc):
        _HEAD_SCALE[0] = self.prev


def _head_scale_buf():
    hs = _HEAD_SCALE[0]
    return hs.buf if hs is not None else None


def note_torch_fallback():
    """A neck / head op ran on torch kernels (called by the fallback branches)."""
    hs = _HEAD_SCALE[0]
    if hs is not None and torch.is_grad_enabled():
        hs.torch_fallback = True


def _unscale_(t, buf):
    """t *= 1/s of a HeadScale buffer (in place, on the device); t may be None."""
    if t is not None and buf is not None:
        t.mul_(buf[1])
    return t


class HeadsOutFn(torch.autograd.Function):
    """The heads' 16-bit low-res outputs as fp32 (what the reference returns for fp32 images);
    backward: the fp32 gradients cast back to the compute dtype, for fp16 with the shared
    power-of-two scale of HeadScale (one s for both heads: their input gradients sum in the
    neck)."""

    @staticmethod
    def forward(ctx, hs, *outs):
        ctx.hs = hs
        ctx.set_materialize_grads(False)  # an unused output's gradient stays None, not zeros
        return tuple(o.float() for o in outs)

    @staticmethod
    def backward(ctx, *gs):
        hs = ctx.hs
        cdt = hs.cdt
        if hs.buf is None or hs.torch_fallback:
            if hs.buf is not None:
                _warn_unscaled_fp16()
            return (None,) + tuple(None if g is None else g.to(cdt) for g in gs)
        live = [g.contiguous() for g in gs if g is not None]
        if not live:
            return (None,) + tuple(None for _ in gs)
        # ONE scale from the joint max |g| of both heads' gradients (they sum in the neck): an
        # all-zero gradient (an empty depth mask, silog weight 0) adds nothing to the maximum,
        # where taking the smaller of two per-head scales let its s = 1 flush the other head's
        # 1e-5..1e-8 gradients in the fp16 cast
        joint = live[0] if len(live) == 1 else torch.cat([g.reshape(-1) for g in live])
        hs.buf.copy_(grad_scale(joint, cdt))
        _stat("head_grad_scale")
        return (None,) + tuple(None if g is None else cast(g.contiguous(), cdt, scale_t=hs.buf) for g in gs)


_WARNED_UNSCALED = [False]


def _warn_unscaled_fp16():
    """A torch fallback op in an fp16 neck / head backward: its gradients run unscaled (s = 1), so
    the 1e-5..1e-8 segmentation gradients may flush to zero in fp16.  Said once, loudly."""
    if not _WARNED_UNSCALED[0]:
        import warnings
        warnings.warn("denseclip: a neck / head op fell back to torch in an fp16 backward; its gradients are "
                      "cast to fp16 without the power-of-two scale and may underflow (use bf16 compute, or a "
                      "config whose neck / heads all run on the HIP kernels)", RuntimeWarning, stacklevel=2)
        _WARNED_UNSCALED[0] = True


def _divides(a, b):
    return b > 0 and a % b == 0


def neck_heads_hip_capable(model):
    """Whether every neck / head op of `model` (a DenseCLIP) has a HIP kernel for 16-bit maps at
    its widths and in its current mode (decided before the backbone runs): the per-level 3x3
    convs (Cin % 128, Cout % 64, concatenated width <= 2048), the 1x1 fusion conv (Cin, Cout %
    64), the BNs (width % 8, <= 2048, a momentum, and training mode whenever a gradient will
    pass them) and the FCN heads (3x3 Cin % 128, 1x1 Cin % 64)."""
    # an eval-mode BN that a gradient must pass (the frozen-BN fine-tune pattern) has no HIP
    # backward (bn_hip_ok: training mode; bn_eval_ok: no gradient), and would fall back to torch
    grads = torch.is_grad_enabled() and any(p.requires_grad for p in model.parameters())

    def bn_ok(bn):
        return (isinstance(bn, torch.nn.BatchNorm2d) and _divides(bn.num_features, 8) and bn.num_features <= 2048
                and bn.affine and bn.track_running_stats and bn.momentum is not None
                and (bn.training or not grads))

    def conv3_ok(conv, cin):
        return (conv.kernel_size == (3, 3) and conv.padding == (1, 1) and conv.stride == (1, 1) and conv.bias is None
                and conv.groups == 1 and conv.dilation == (1, 1) and _divides(cin, 128) and conv.in_channels == cin)

    width = getattr(model.backbone, "width", None)
    if width is None:
        return False
    head_in = width
    neck = model.neck
    if neck is not None:
        layers = list(neck.process_layers)
        if not layers:
            return False
        Ci = layers[0][0].out_channels
        for layer in layers:
            if not (conv3_ok(layer[0], width) and layer[0].out_channels == Ci and bn_ok(layer[1])):
                return False
        if not (_divides(Ci, 64) and len(layers) * Ci <= 2048):
            return False
        fconv, fbn = neck.fusion_layer[0], neck.fusion_layer[1]
        if not (fconv.kernel_size == (1, 1) and fconv.stride == (1, 1) and fconv.groups == 1
                and _divides(fconv.in_channels, 64) and _divides(fconv.out_channels, 64) and bn_ok(fbn)):
            return False
        head_in = fconv.out_channels
    for head in (model.decode_head, model.depth_head):
        if head is None:
            continue
        if len(head) != 6:
            return False
        c3, bn, _, _, c1, cl = head
        if not (conv3_ok(c3, head_in) and bn_ok(bn) and c1.kernel_size == (1, 1) and cl.kernel_size == (1, 1)
                and c1.bias is not None and cl.bias is not None and c1.stride == (1, 1) and cl.stride == (1, 1)
                and c1.groups == 1 and cl.groups == 1 and _divides(c1.in_channels, 64)):
            return False
    return model.decode_head is not None or model.depth_head is not None


# ============================================================================ neck convs
def _pad64(n):
    return (n + 63) // 64 * 64


def pixel_rows(xmap, cdt):
    """Channels-last pixel-row geometry of an NCHW-shaped map (B, C, H, W): returns
    (tensor whose data_ptr is pixel (0, 0, 0), batch stride, pixel pitch), all in elements.
    Token-buffer views (ReadoutFn) and channels_last tensors are used in place; anything
    else gets one NHWC copy."""
    B, C, H, W = xmap.shape
    st = xmap.stride()
    if xmap.dtype == cdt and st[1] == 1 and st[3] == C and st[2] == W * C and st[0] % 8 == 0 and C % 8 == 0 \
            and xmap.data_ptr() % 16 == 0:
        return xmap, st[0], C
    xr = xmap.to(cdt).permute(0, 2, 3, 1).contiguous()
    return xr, H * W * C, C


def conv3x3_fwd(xmap, w_rows, cout_pad, cdt):
    """out (B*H*W, cout_pad) = 3x3 / pad 1 conv of xmap with w_rows (cout_pad, 9*Cin) in
    (ky, kx, ci) order (models.py:741-745 via ConvBNReLU, 13-20)."""
    B, Cin, H, W = xmap.shape
    xr, bs, ld = pixel_rows(xmap, cdt)
    _check(w_rows, strided=(xr,))
    out = torch.empty(B * H * W, cout_pad, dtype=cdt, device=xmap.device)
    D().conv3x3(0, xr, bs, 0, ld, B, H, W, Cin, w_rows, cout_pad, out, cout_pad, 0, 0, 0)
    return out, (xr, bs, ld)


class Conv3x3Fn(torch.autograd.Function):
    """3x3 / stride 1 / pad 1 convolution without bias (the neck's per-level conv,
    reference models.py:17 inside ConvBNReLU, models.py:741-745) as implicit MFMA GEMMs on
    channels-last pixel rows: forward, input gradient (dgrad) and weight gradient (wgrad).
    Returns a channels-last (B, Cout, H, W) tensor.  The input gradient has the input's own
    layout (for a ViT token-buffer view: a token buffer whose CLS rows are zero), which
    ReadoutFn.backward takes without a copy."""

    @staticmethod
    def forward(ctx, xmap, weight, cdt):
        B, Cin, H, W = xmap.shape
        Cout = weight.shape[0]
        cp = _pad64(Cout)

        w_rows = _conv3x3_rows(weight, cdt)
        out, (xr, bs, ld) = conv3x3_fwd(xmap, w_rows, cp, cdt)
        ctx.save_for_backward(xr, weight)
        ctx.geo = (B, Cin, H, W, Cout, cp, bs, ld, xmap.dtype, tuple(xmap.stride()), xmap.storage_offset() -
                   (xr.storage_offset() if xr is xmap else 0), xr is xmap)
        ctx.cdt = cdt
        ctx.hsb = _head_scale_buf()
        _stat("conv3x3")
        y = out.as_strided((B, Cout, H, W), (H * W * cp, 1, W * cp, cp))
        return y

    @staticmethod
    def backward(ctx, dy):
        xr, weight = ctx.saved_tensors
        B, Cin, H, W, Cout, cp, bs, ld, in_dt, in_strides, _, in_place = ctx.geo
        cdt = ctx.cdt
        M = B * H * W
        dyr = torch.zeros(M, cp, dtype=cdt, device=dy.device)
        dyr[:, :Cout] = dy.permute(0, 2, 3, 1).reshape(M, Cout)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            w_t = _conv3x3_dgrad_rows(weight, cdt)
            if in_place and in_strides[0] == bs:
                # same layout as the input view: batches of bs elements, pixel rows after a gap
                gap_rows = (bs - H * W * ld) // ld
                # the gap (CLS) rows stay unwritten: every reader of this token-layout gradient skips
                # or overwrites them (dclip_add_readout_cast, BlockFn / ReadoutFn's CLS masking)
                buf = torch.empty(B * bs, dtype=cdt, device=dy.device)
                D().conv3x3(1, dyr, H * W * cp, 0, cp, B, H, W, cp, w_t, Cin, buf, ld, gap_rows, gap_rows, 0)
                dx = buf.as_strided((B, Cin, H, W), (bs, 1, W * ld, ld), gap_rows * ld)
            else:
                buf = torch.empty(M, Cin, dtype=cdt, device=dy.device)
                D().conv3x3(1, dyr, H * W * cp, 0, cp, B, H, W, cp, w_t, Cin, buf, Cin, 0, 0, 0)
                dx = buf.as_strided((B, Cin, H, W), (H * W * Cin, 1, W * Cin, Cin))
            if in_dt != cdt:
                dx = dx.to(in_dt)
        if ctx.needs_input_grad[1]:
            tiles = (cp + 127) // 128 * (9 * Cin // 128)
            splits = max(1, min(32, 512 // max(1, tiles), M // 4096 or 1))
            e0 = _tic()
            # torch's (Cout, Cin, 3, 3) layout and the heads' 1/s straight out of the split-K sum
            dw = D().conv3x3_wgrad(dyr, cp, cp, xr, bs, 0, ld, B, H, W, Cin, splits, True, ctx.hsb)
            _toc("conv_wgrad", e0)
            dw = dw[:Cout]
            if dw.dtype != weight.dtype:
                dw = dw.to(weight.dtype)
        return dx, dw, None


def _conv3x3_rows(weight, cdt):
    """(Cout, Cin, 3, 3) -> cached (cp, 9*Cin) rows in (ky, kx, ci) order, zero rows past Cout.
    Cout % 64 == 0 (every conv of the Cityscapes configs): one batched transpose launch
    (per output channel, (Cin, 9) -> (9, Cin), cast on the fly) instead of a permute copy and a
    cast copy."""
    Cout, Cin = weight.shape[:2]
    cp = _pad64(Cout)

    def rows(w):
        if cp == Cout and w.is_cuda:
            return D().transpose_batched(w.contiguous(), Cout, Cin, 9, 9, Cin, cdt).view(Cout, 9 * Cin)
        r = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)
        return torch.cat([r, r.new_zeros(cp - Cout, 9 * Cin)]) if cp > Cout else r
    return WEIGHTS.get_with(weight, cdt, "conv3x3_rows", rows)


def _conv3x3_dgrad_rows(weight, cdt):
    """(Cout, Cin, 3, 3) -> cached (Cin, 9*cp): [ci][tap][co], zero columns past Cout.  For
    Cout % 64 == 0 this is the plain transposed weight copy ((Cout, 9 Cin) -> (9 Cin, Cout), the
    16-byte transpose kernel) viewed as (Cin, 9 Cout)."""
    Cout, Cin = weight.shape[:2]
    cp = _pad64(Cout)
    if cp == Cout and weight.is_cuda:
        return WEIGHTS.get(weight, cdt, transposed=True).view(Cin, 9 * cp)

    def trows(w):
        t = w.permute(1, 2, 3, 0)
        if cp > Cout:
            t = torch.cat([t, t.new_zeros(Cin, 3, 3, cp - Cout)], dim=3)
        return t.reshape(Cin, 9 * cp)
    return WEIGHTS.get_with(weight, cdt, "conv3x3_dgrad", trows)


class NeckLevelsFn(torch.autograd.Function):
    """The fusion neck's per-level ConvModules + concatenation (reference models.py:741-765:
    12 x [3x3 conv C -> Ci, BN, ReLU], torch.cat over channels) in train mode, without the
    concatenation copy: level l's implicit-GEMM conv writes its Ci channels straight into columns
    [l*Ci, (l+1)*Ci) of one (B*H*W, L*Ci) pre-activation buffer, and its BN + ReLU (batch
    statistics, fused) writes the same columns of the concatenated output, which the 1x1 fusion
    conv reads as it is.  The backward runs the same way on column slices: fused BN + ReLU
    backward per level into a dgrad buffer whose slices feed each level's dgrad / wgrad convs.
    Inputs: L maps (channels-last views, e.g. token-buffer read-outs), then per level the conv
    weight, BN weight, BN bias; the BN modules are in meta (running statistics updated in place)."""

    @staticmethod
    def forward(ctx, meta, *args):
        bns, cdt = meta
        L = len(bns)
        maps = args[:L]
        convw = args[L:2 * L]
        bnw = args[2 * L:3 * L]
        bnb = args[3 * L:4 * L]
        B, Cin, H, W = maps[0].shape
        Ci = convw[0].shape[0]
        M, LC = B * H * W, L * Ci
        pre = torch.empty(M, LC, dtype=cdt, device=maps[0].device)
        out = torch.empty(M, LC, dtype=cdt, device=maps[0].device)
        geo, stats = [], []
        for l in range(L):
            xr, bs, ld = pixel_rows(maps[l], cdt)
            D().conv3x3(0, xr, bs, 0, ld, B, H, W, Cin, _conv3x3_rows(convw[l], cdt), Ci, pre[:, l * Ci:], LC, 0, 0, 0)
            bn = bns[l]
            if bn.num_batches_tracked is not None:
                bn.num_batches_tracked.add_(1)
            mean, rstd = D().bn_fwd_rows(pre[:, l * Ci:(l + 1) * Ci], bnw[l].detach(), bnb[l].detach(), bn.running_mean,
                                         bn.running_var, float(bn.momentum), float(bn.eps), True,
                                         out[:, l * Ci:(l + 1) * Ci])
            geo.append((xr, bs, ld))
            stats += [mean, rstd]
        ctx.save_for_backward(pre, *[g[0] for g in geo], *convw, *bnw, *bnb, *stats)
        ctx.meta = (L, B, Cin, H, W, Ci, cdt, [(g[1], g[2]) for g in geo], [m.dtype for m in maps],
                    [tuple(m.stride()) for m in maps], [g[0] is m for g, m in zip(geo, maps)])
        ctx.hsb = _head_scale_buf()
        ctx.links = [getattr(m, "_dclip_link", None) for m in maps]  # ReadoutLink of a block's map
        _stat("neck_levels")
        return out.as_strided((B, LC, H, W), (H * W * LC, 1, W * LC, LC))

    @staticmethod
    def backward(ctx, dout):
        L, B, Cin, H, W, Ci, cdt, bsld, in_dts, in_strides, in_place = ctx.meta
        saved = ctx.saved_tensors
        pre = saved[0]
        xrs = saved[1:1 + L]
        convw = saved[1 + L:1 + 2 * L]
        bnw = saved[1 + 2 * L:1 + 3 * L]
        bnb = saved[1 + 3 * L:1 + 4 * L]
        stats = saved[1 + 4 * L:]
        M, LC = B * H * W, L * Ci
        d = dout.to(cdt).permute(0, 2, 3, 1).reshape(M, LC)
        if not d.is_contiguous():
            d = d.contiguous()
        dpre = torch.empty(M, LC, dtype=cdt, device=d.device)
        need = ctx.needs_input_grad  # (meta, maps..., convw..., bnw..., bnb...)
        dmaps, dconv, dbnw, dbnb = [None] * L, [None] * L, [None] * L, [None] * L
        tiles = (Ci + 127) // 128 * (9 * Cin // 128)
        splits = max(1, min(32, 512 // max(1, tiles), M // 4096 or 1))
        for l in range(L):
            sl = slice(l * Ci, (l + 1) * Ci)
            dbnw[l], dbnb[l] = D().bn_bwd_rows(d[:, sl], pre[:, sl], bnw[l].detach(), bnb[l].detach(), stats[2 * l],
                                               stats[2 * l + 1], True, True, True, dpre[:, sl], ctx.hsb)
            bs, ld = bsld[l]
            if need[1 + l]:  # input gradient: the dgrad conv, in the input's own layout when it is a token view
                w_t = _conv3x3_dgrad_rows(convw[l], cdt)
                if in_place[l] and in_strides[l][0] == bs:
                    gap_rows = (bs - H * W * ld) // ld
                    buf = torch.empty(B * bs, dtype=cdt, device=d.device)  # CLS rows unread (see Conv3x3Fn)
                    D().conv3x3(1, dpre[:, l * Ci:], H * W * LC, 0, LC, B, H, W, Ci, w_t, Cin, buf, ld, gap_rows,
                                gap_rows, 0)
                    dm = buf.as_strided((B, Cin, H, W), (bs, 1, W * ld, ld), gap_rows * ld)
                else:
                    buf = torch.empty(M, Cin, dtype=cdt, device=d.device)
                    D().conv3x3(1, dpre[:, l * Ci:], H * W * LC, 0, LC, B, H, W, Ci, w_t, Cin, buf, Cin, 0, 0, 0)
                    dm = buf.as_strided((B, Cin, H, W), (H * W * Cin, 1, W * Cin, Cin))
                dmaps[l] = dm if in_dts[l] == cdt else dm.to(in_dts[l])
                if ctx.links[l] is not None:
                    ctx.links[l].g = dmaps[l]
            if need[1 + L + l]:
                e0 = _tic()
                dwc = D().conv3x3_wgrad(dpre[:, l * Ci:], LC, Ci, xrs[l], bs, 0, ld, B, H, W, Cin, splits, True, ctx.hsb)
                _toc("conv_wgrad", e0)
                dconv[l] = dwc if dwc.dtype == convw[l].dtype else dwc.to(convw[l].dtype)
        return (None, *dmaps, *dconv, *dbnw, *dbnb)


def neck_levels_hip_ok(layers, feats):
    """Every level a 3x3 ConvModule with a train-mode BN the HIP kernels take, 16-bit GPU maps
    of one shape, Cin % 128 == 0, Ci % 8 == 0 and Ci <= 2048 / levels."""
    if not feats or not all(f.is_cuda and f.dim() == 4 and f.dtype in (torch.bfloat16, torch.float16) for f in feats):
        return False
    if len({(tuple(f.shape), f.dtype) for f in feats}) != 1:
        return False
    Ci = layers[0][0].weight.shape[0]
    for layer in layers:
        conv, bn = layer[0], layer[1]
        if conv.kernel_size != (3, 3) or conv.bias is not None or conv.weight.shape[0] != Ci or \
                not conv3x3_supported(feats[0], conv.weight):
            return False
        f32 = all(t is not None and t.dtype == torch.float32 for t in (bn.weight, bn.bias, bn.running_mean,
                                                                       bn.running_var))
        if not (bn.training and bn.track_running_stats and bn.momentum is not None and f32):
            return False
    return Ci % 64 == 0 and len(layers) * Ci <= 2048


def conv3x3_supported(xmap, weight):
    return (xmap.is_cuda and xmap.dim() == 4 and weight.shape[2:] == (3, 3) and xmap.shape[1] % 128 == 0
            and weight.shape[1] == xmap.shape[1])


class Conv1x1Fn(torch.autograd.Function):
    """1x1 convolution with optional bias on a channels-last map (the neck's fusion conv,
    reference models.py:750 via ConvBNReLU) as one MFMA GEMM over pixel rows; gradients by
    the NT GEMM (input) and the TN weight-gradient GEMM."""

    @staticmethod
    def forward(ctx, xmap, weight, bias, cdt):
        B, Cin, H, W = xmap.shape
        Cout = weight.shape[0]
        # (B*H*W, Cin) pixel rows: a view of a channels-last map, else one NHWC copy
        x2 = xmap.to(cdt).permute(0, 2, 3, 1).reshape(B * H * W, Cin).contiguous()
        out = gemm(x2, WEIGHTS.get(weight, cdt), bias=bias.detach() if bias is not None else None)
        ctx.save_for_backward(x2, weight)
        ctx.meta = (B, Cin, H, W, Cout, bias is not None, xmap.dtype)
        ctx.cdt = cdt
        ctx.hsb = _head_scale_buf()
        _stat("conv1x1")
        return out.as_strided((B, Cout, H, W), (H * W * Cout, 1, W * Cout, Cout))

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        B, Cin, H, W, Cout, has_b, in_dt = ctx.meta
        cdt = ctx.cdt
        d2 = dy.permute(0, 2, 3, 1).reshape(B * H * W, Cout)
        d2 = d2.to(cdt).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gemm(d2, WEIGHTS.get(weight, cdt, transposed=True))
            dx = dx.as_strided((B, Cin, H, W), (H * W * Cin, 1, W * Cin, Cin))
            if in_dt != cdt:
                dx = dx.to(in_dt)
        if ctx.needs_input_grad[1] or (has_b and ctx.needs_input_grad[2]):
            dWm, dbm = weight_grad(d2, x2, want_bias=has_b, scale=ctx.hsb)
            dw = dWm.view_as(weight).to(weight.dtype)
            db = dbm
        return dx, dw, db, None


def conv1x1_supported(xmap, weight):
    return (xmap.is_cuda and xmap.dim() == 4 and weight.shape[2:] == (1, 1) and xmap.shape[1] % 64 == 0
            and weight.shape[0] % 64 == 0)  # K of the forward and of the input-gradient GEMM


# ============================================================================ FCN heads
def _merged_tail(w1, b1, wc, bc, cdt, Kp):
    """The merged head tail (Kp x Cin weight Wc W1 in cdt, zero rows past K; f32 bias Wc b1 + bc),
    cached on the classifier weight until any of the four parameters changes (the weight cache's
    stamps: optimizer step, version, storage) — not recomputed by torch matmuls every forward."""
    stamp = (cdt, Kp) + tuple(_Cast.stamp(p) for p in (w1, b1, wc, bc))
    ent = wc.__dict__.get("_dclip_merged")
    if ent is not None and ent[0] == stamp:
        return ent[1], ent[2]
    C1, Cin, K = w1.shape[0], w1.shape[1], wc.shape[0]
    with torch.autocast("cuda", enabled=False), torch.no_grad():
        W1m = w1.detach().reshape(C1, Cin).float()
        Wcm = wc.detach().reshape(K, C1).float()
        Wp = torch.zeros(Kp, Cin, dtype=cdt, device=w1.device)
        Wp[:K] = Wcm @ W1m
        bp = torch.zeros(Kp, dtype=torch.float32, device=w1.device)
        bp[:K] = Wcm @ b1.detach().float() + bc.detach().float()
    wc.__dict__["_dclip_merged"] = (stamp, Wp, bp)
    return Wp, bp


class MergedPointwiseFn(torch.autograd.Function):
    """The FCN head's tail — 1x1 conv (Cin -> C1, bias) then the classifier 1x1 conv (C1 -> K,
    bias) (torchvision FCNHead + DenseCLIP's classifier, reference denseclip.py:305-309,
    343-349) — as ONE MFMA GEMM with the merged weight Wc W1 (K x Cin) and bias Wc b1 + bc: the
    (B, C1, H, W) intermediate never exists.  The backward needs it only through
    dWc = dY^T h = (dY^T X) W1^T + colsum(dY) b1^T, so it runs two K-row GEMMs on the pixel rows
    (dX, and dY^T X by the TN weight-gradient GEMM) and tiny K x Cin products.  Output: NCHW
    (B, K, H, W) in the compute dtype (the head's logits)."""

    @staticmethod
    def forward(ctx, y, w1, b1, wc, bc, cdt):
        B, Cin, H, W = y.shape
        C1, K = w1.shape[0], wc.shape[0]
        Kp = _pad64(K)
        Wp, bp = _merged_tail(w1, b1, wc, bc, cdt, Kp)
        y2 = y.to(cdt).permute(0, 2, 3, 1).reshape(B * H * W, Cin)
        if not y2.is_contiguous():
            y2 = y2.contiguous()
        rows = gemm(y2, Wp, bias=bp)  # (B*H*W, Kp)
        out = D().transpose_batched(rows, B, H * W, K, Kp, H * W, cdt)  # (B, K, H*W)
        ctx.save_for_backward(y2, w1, b1, wc, Wp)
        ctx.meta = (B, Cin, H, W, C1, K, Kp, y.dtype, cdt)
        ctx.hsb = _head_scale_buf()
        _stat("merged_pointwise")
        return out.view(B, K, H, W)

    @staticmethod
    def backward(ctx, dout):
        y2, w1, b1, wc, Wp = ctx.saved_tensors
        B, Cin, H, W, C1, K, Kp, in_dt, cdt = ctx.meta
        dY = D().transpose_batched(dout.contiguous(), B, K, H * W, H * W, Kp, cdt).view(B * H * W, Kp)
        need = ctx.needs_input_grad
        dy = None
        if need[0]:
            dX = gemm(dY, transpose2d(Wp, cdt))  # (B*H*W, Cin)
            dy = dX.as_strided((B, Cin, H, W), (H * W * Cin, 1, W * Cin, Cin))
            if in_dt != cdt:
                dy = dy.to(in_dt)
        dw1 = db1 = dwc = dbc = None
        if any(need[1:5]):
            G, cs = weight_grad(dY, y2, scale=ctx.hsb)  # (Kp, Cin) = dY^T X, colsum(dY), unscaled
            with torch.autocast("cuda", enabled=False):
                G, cs = G[:K], cs[:K]
                W1m = w1.detach().reshape(C1, Cin).float()
                Wcm = wc.detach().reshape(K, C1).float()
                dwc = (G @ W1m.t() + cs[:, None] * b1.detach().float()[None, :]).reshape(wc.shape).to(wc.dtype)
                dw1 = (Wcm.t() @ G).reshape(w1.shape).to(w1.dtype)
                db1 = (Wcm.t() @ cs).to(b1.dtype)
                dbc = cs.to(wc.dtype)
        return dy, dw1, db1, dwc, dbc, None


def fcn_head_hip_ok(head, x):
    """FCNHead + classifier in the layout DenseCLIP builds (conv3x3 no-bias, BN, ReLU, Dropout,
    conv1x1 + bias, classifier conv1x1 + bias) on a 16-bit GPU map."""
    if len(head) != 6 or not (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float16)):
        return False
    c3, _, _, _, c1, cl = head
    return (c3.kernel_size == (3, 3) and c3.padding == (1, 1) and c3.stride == (1, 1) and c3.bias is None
            and c1.kernel_size == (1, 1) and cl.kernel_size == (1, 1) and c1.bias is not None and cl.bias is not None
            and c1.stride == (1, 1) and cl.stride == (1, 1) and c1.weight.shape[1] % 64 == 0
            and conv3x3_supported(x, c3.weight) and c1.groups == 1 and cl.groups == 1)


def fcn_head(head, x):
    """FCNHead forward on the HIP kernels: implicit-GEMM 3x3 conv, BN + ReLU (batch statistics
    in train mode; torch's eval BN otherwise), Dropout (torch), merged 1x1 tail."""
    c3, bn, relu, drop, c1, cl = head
    cdt = x.dtype
    _stat("fcn_head")
    y = Conv3x3Fn.apply(x, c3.weight, cdt)
    if bn_hip_ok(bn, y):
        y = bn_train(bn, y, relu=True)
    elif bn_eval_ok(bn, y):
        y = bn_eval(bn, y, relu=True)
    else:
        note_torch_fallback()
        y = relu(bn(y))
    y = drop(y)
    return MergedPointwiseFn.apply(y, c1.weight, c1.bias, cl.weight, cl.bias, cdt)


# ============================================================================ fused head losses
_LAB_DT = {torch.int64: 0, torch.int32: 1, torch.uint8: 2}


class UpsampleCEFn(torch.autograd.Function):
    """F.cross_entropy(F.interpolate(logits, (H, W), bilinear, align_corners=False), labels,
    ignore_index) (reference denseclip.py:847 resize + train_denseclip.py:1265-1314 CE) in one
    pass over the labels: the upsampled logits are never materialised; the gradient wrt the
    low-res logits is produced in the same pass (scaled by grad / #valid in backward)."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        B, K, h, w = logits.shape
        H, W = labels.shape[-2:]
        lg = logits.detach().contiguous()
        lab = labels.contiguous()
        _check(lg, lab)
        if lab.dtype not in _LAB_DT:
            lab = lab.long()
        e0 = _tic()
        sums, cnt, grad = D().upsample_ce(lg, lab, int(ignore_index))
        _toc("upsample_ce", e0)
        n = cnt.to(torch.float64).clamp(min=1)
        ctx.save_for_backward(grad, n)
        ctx.in_dtype = logits.dtype
        # all labels ignored: NaN, like torch's CrossEntropyLoss (0 / 0); no host sync
        mean = torch.where(cnt > 0, sums / n, torch.full_like(sums, float("nan")))
        return mean.to(torch.float32).reshape(())

    @staticmethod
    def backward(ctx, g):
        grad, n = ctx.saved_tensors
        d = grad * (g.to(torch.float64) / n).to(torch.float32)
        return d.to(ctx.in_dtype), None, None


class UpsampleSILogFn(torch.autograd.Function):
    """SILogLoss(lambd, eps)(F.interpolate(pred, (H, W), bilinear, align_corners=False),
    target, mask) (reference losses.py:21-78 on the resized depth, denseclip.py:860) without
    materialising the resized prediction: a sums pass in forward, a gradient pass in backward."""

    @staticmethod
    def forward(ctx, pred, target, mask, lambd, eps):
        B, _, h, w = pred.shape
        H, W = target.shape[-2:]
        pd = pred.detach().contiguous()
        tg = target.detach().reshape(B, H, W).float().contiguous()
        mk = mask.reshape(B, H, W).to(torch.uint8).contiguous() if mask is not None else None
        _check(pd, tg, mk)
        sums = D().upsample_silog_sums(pd, tg, mk, float(eps))
        T = sums[2].clamp(min=1)
        loss = sums[1] / T - lambd * sums[0] ** 2 / T ** 2
        loss = torch.where(sums[2] > 0, loss, torch.zeros_like(loss))
        ctx.save_for_backward(pd, tg, mk, sums)
        ctx.args = (lambd, eps, pred.dtype)
        return loss.to(torch.float32)

    @staticmethod
    def backward(ctx, g):
        pd, tg, mk, sums = ctx.saved_tensors
        lambd, eps, in_dtype = ctx.args
        grad = D().upsample_silog_grad(pd, tg, mk, sums, float(eps), float(lambd))
        return (grad * g.to(torch.float32)).to(in_dtype), None, None, None, None
