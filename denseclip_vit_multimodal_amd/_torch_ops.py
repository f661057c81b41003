"""torch.ops.dclip.*: the TORCH_LIBRARY custom ops of libdclip_torch.so (csrc/torch_ops.cpp, an
adapter over the C ABI of include/dclip.h) and their fake (meta) implementations, so the ops
trace under torch.compile / torch.export / FakeTensorMode and pass torch.library.opcheck.

There is no CPU kernel: a CPU tensor reaching an op raises (NotImplementedError from the
dispatcher for the CPU key), and a missing library raises at import.
"""
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DCLIP_TORCH_LIB", os.path.join(_HERE, "libdclip_torch.so"))

_loaded = False


def load():
    """Load libdclip_torch.so into the torch dispatcher once (it links libdclip.so)."""
    global _loaded
    if _loaded:
        return torch.ops.dclip
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libdclip_torch.so not found at {LIB_PATH}: build it with "
                           "`make -C denseclip_vit_multimodal_amd/csrc` (the HIP path has no CPU fallback)")
    from . import _native
    # libdclip_torch.so binds the libdclip.so next to it (rpath $ORIGIN): a DCLIP_LIB pointing at
    # another build would be configured (dclip_set_option) while every op ran the other one
    bound = os.path.realpath(os.path.join(os.path.dirname(LIB_PATH), "libdclip.so"))
    if os.path.realpath(_native.LIB_PATH) != bound:
        raise RuntimeError(f"DCLIP_LIB ({_native.LIB_PATH}) is not the libdclip.so that {LIB_PATH} binds ({bound}); "
                           "build a matching adapter and point DCLIP_TORCH_LIB at it")
    _native.load()  # same libdclip.so instance (DCLIP_OPTIONS are applied there)
    torch.ops.load_library(LIB_PATH)
    _register_fakes()
    _loaded = True
    return torch.ops.dclip


def _e(*shape, like, dtype=None):
    return like.new_empty(shape, dtype=dtype if dtype is not None else like.dtype)


def _register_fakes():
    reg = torch.library.register_fake
    f32 = torch.float32

    @reg("dclip::layernorm_fwd")
    def _(x, w, b, out_dtype, eps):
        r, c = x.shape
        return _e(r, c, like=x, dtype=out_dtype), _e(r, like=x, dtype=f32), _e(r, like=x, dtype=f32)

    @reg("dclip::layernorm_bwd")
    def _(dy, x, w, mean, rstd, res, dw, db, dy_scale=None, dy_ntok=0):
        return _e(*x.shape, like=x, dtype=f32)

    @reg("dclip::layernorm_bwd_lp")
    def _(dy, x, w, mean, rstd, res, dw, db, lp_dtype, dy_scale=None):
        return _e(*x.shape, like=x, dtype=f32), _e(*x.shape, like=x, dtype=lp_dtype)

    @reg("dclip::layernorm_bwd_add")
    def _(dy, x, w, mean, rstd, res, add, ntok, dw, db, lp_dtype):
        return _e(*x.shape, like=x, dtype=f32), _e(*x.shape, like=x, dtype=lp_dtype)

    @reg("dclip::gemm")
    def _(A, B, epi, bias, aux, out_dtype, alpha, scale=None):
        return _e(A.shape[0], B.shape[0], like=A, dtype=out_dtype)

    @reg("dclip::gemm_gelu")
    def _(A, B, bias):
        return _e(A.shape[0], B.shape[0], like=A), _e(A.shape[0], B.shape[0], like=A)

    @reg("dclip::gemm_gelu_h")
    def _(A, B, bias):
        return _e(A.shape[0], B.shape[0], like=A)

    @reg("dclip::gemm_residual_lp")
    def _(A, B, bias, aux):
        return _e(A.shape[0], B.shape[0], like=A, dtype=f32), _e(A.shape[0], B.shape[0], like=A)

    @reg("dclip::weight_grad")
    def _(dy, x, alpha, db, scale=None):
        return _e(dy.shape[1], x.shape[1], like=dy, dtype=f32)

    @reg("dclip::gemm_tn")
    def _(A, B):
        return _e(A.shape[1], B.shape[1], like=A, dtype=f32)

    @reg("dclip::cast")
    def _(x, dtype, scale, scale_t=None):
        return _e(*x.shape, like=x, dtype=dtype)

    @reg("dclip::bn_eval")
    def _(x, w, b, running_mean, running_var, eps, relu):
        return torch.empty_like(x, memory_format=torch.channels_last)

    @reg("dclip::row_scale_add")
    def _(x, y, s):
        return torch.empty_like(y)

    @reg("dclip::grad_scale")
    def _(g, target):
        return _e(4, like=g, dtype=f32)

    @reg("dclip::transpose2d")
    def _(x, dtype):
        return _e(x.shape[1], x.shape[0], like=x, dtype=dtype)

    @reg("dclip::weight_refresh")
    def _(desc, tiles, dtype):
        return None

    @reg("dclip::transpose_batched")
    def _(x, B, rows, cols, ld_in, rows_pad, dtype):
        return _e(B, cols, rows_pad, like=x, dtype=dtype)

    @reg("dclip::add_readout_cast")
    def _(a, b, ntok, lp_dtype, scale):
        return _e(*a.shape, like=a), _e(*a.shape, like=a, dtype=lp_dtype)

    @reg("dclip::add_readout_amax")
    def _(a, b, ntok, b_scale, target):
        return _e(*a.shape, like=a), _e(4, like=a)

    @reg("dclip::add_readout_cast_scaled")
    def _(a, b, ntok, b_scale, st, use, target):
        return (_e(*a.shape, like=a) if b is not None else _e(0, like=a)), _e(*a.shape, like=a, dtype=torch.float16), _e(4, like=a)

    @reg("dclip::layernorm_bwd_scaled")
    def _(dy, x, w, mean, rstd, res, dw, db, st, use, target, dy_scale=None):
        return _e(*x.shape, like=x, dtype=f32), _e(*x.shape, like=x, dtype=torch.float16), _e(4, like=x)

    @reg("dclip::layernorm_bwd_scaled_add")
    def _(dy, x, w, mean, rstd, res, add, add_scale, ntok, dw, db, st, use, target, dy_scale=None):
        return _e(*x.shape, like=x, dtype=f32), _e(*x.shape, like=x, dtype=torch.float16), _e(4, like=x)

    @reg("dclip::attn_fwd")
    def _(qkv, B, N, H, scale):
        return _e(B * N, 64 * H, like=qkv), _e(B * H * N, like=qkv, dtype=f32)

    @reg("dclip::attn_fwd_fp8")
    def _(qkv, B, N, H):
        return _e(B * N, 64 * H, like=qkv), _e(B * H * N, like=qkv, dtype=f32)

    @reg("dclip::attn_bwd")
    def _(qkv, o, dout, lse, B, N, H, scale):
        return torch.empty_like(qkv)

    @reg("dclip::attn_bwd_fp8")
    def _(qkv, o, dout, lse, B, N, H, scale):
        return torch.empty_like(qkv)

    @reg("dclip::im2col")
    def _(img, p, dtype):
        B, Cin, Hi, Wi = img.shape
        return _e(B * (Hi // p) * (Wi // p), -(-Cin * p * p // 64) * 64, like=img, dtype=dtype)

    @reg("dclip::tokens_fwd")
    def _(emb, cls, pos, B, P):
        return _e(B * (P + 1), emb.shape[1], like=emb, dtype=f32)

    @reg("dclip::tokens_bwd")
    def _(dx, dtype, scale, B, P, scale_t=None):
        C = dx.shape[1]
        return _e(B * P, C, like=dx, dtype=dtype), _e(C, like=dx, dtype=f32), _e(P + 1, C, like=dx, dtype=f32)

    @reg("dclip::pos_interp")
    def _(pos, g, H, W):
        return _e(H * W + 1, pos.shape[1], like=pos)

    @reg("dclip::pos_interp_bwd")
    def _(dout, g, H, W):
        return _e(g * g + 1, dout.shape[1], like=dout)

    @reg("dclip::row_mean")
    def _(x, bstride, row_off, ld, B, rows, C):
        return _e(B, C, like=x, dtype=f32)

    @reg("dclip::score_map")
    def _(v, bstride, row_off, ld, text, B, HW, eps):
        return _e(B, text.shape[1], HW, like=v, dtype=f32)

    @reg("dclip::score_concat")
    def _(rows, bstride, row_off, ld, C, score, B, h, w):
        return _e(B * h * w, C + score.shape[1], like=rows)

    @reg("dclip::bilinear")
    def _(x, Ho, Wo, dtype):
        return _e(x.shape[0], x.shape[1], Ho, Wo, like=x, dtype=dtype)

    @reg("dclip::bilinear_bwd")
    def _(dout, Hi, Wi):
        return _e(dout.shape[0], dout.shape[1], Hi, Wi, like=dout, dtype=f32)

    @reg("dclip::bn_fwd")
    def _(x, w, b, running_mean, running_var, momentum, eps, relu):
        C = x.shape[1]
        return (torch.empty_like(x, memory_format=torch.channels_last), _e(C, like=x, dtype=f32),
                _e(C, like=x, dtype=f32))

    @reg("dclip::bn_bwd")
    def _(dy, x, w, b, mean, rstd, relu, want_w, want_b, scale=None):
        C = x.shape[1]
        return (torch.empty_like(x, memory_format=torch.channels_last), _e(C if want_w else 0, like=x, dtype=f32),
                _e(C if want_b else 0, like=x, dtype=f32))

    @reg("dclip::bn_fwd_rows")
    def _(x, w, b, running_mean, running_var, momentum, eps, relu, y):
        return _e(x.shape[1], like=x, dtype=f32), _e(x.shape[1], like=x, dtype=f32)

    @reg("dclip::bn_bwd_rows")
    def _(dy, x, w, b, mean, rstd, relu, want_w, want_b, dx, scale=None):
        C = x.shape[1]
        return _e(C if want_w else 0, like=x, dtype=f32), _e(C if want_b else 0, like=x, dtype=f32)

    @reg("dclip::conv3x3")
    def _(mode, X, x_bstride, x_off, x_ld, B, H, W, Cin, Wt, Nout, out, out_ld, out_gap, out_off, accumulate):
        return None

    @reg("dclip::conv3x3_wgrad")
    def _(dY, ldy, Nout, X, x_bstride, x_off, x_ld, B, H, W, Cin, splits, oihw=False, scale=None):
        return _e(Nout, Cin, 3, 3, like=X, dtype=f32) if oihw else _e(Nout, 9 * Cin, like=X, dtype=f32)

    @reg("dclip::upsample_ce")
    def _(logits, labels, ignore_index):
        return (_e(1, like=logits, dtype=torch.float64), _e(1, like=logits, dtype=torch.int32),
                _e(*logits.shape, like=logits, dtype=f32))

    @reg("dclip::upsample_silog_sums")
    def _(pred, target, mask, eps):
        return _e(3, like=pred, dtype=torch.float64)

    @reg("dclip::upsample_silog_grad")
    def _(pred, target, mask, sums, eps, lambd):
        return _e(*pred.shape, like=pred, dtype=f32)

    @reg("dclip::cityscapes_prepare")
    def _(img, ids, disp, crop, h, w, mean, std, bf, depth_max, out_dtype, jitter=None):
        B = img.shape[0]
        return (_e(B, 3, h, w, like=img, dtype=out_dtype), _e(B, h, w, like=img, dtype=torch.int64),
                _e(B, 1, h, w, like=img, dtype=f32), _e(B, 1, h, w, like=img, dtype=torch.uint8))
