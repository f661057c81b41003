"""The TORCH_LIBRARY(dclip) surface (csrc/torch_ops.cpp over the C ABI) without a GPU: every op
is registered with its schema, the fake (meta) implementations give the shapes / dtypes the
HIP kernels produce (so the ops trace under FakeTensorMode / torch.compile), and a CPU tensor
is refused by the dispatcher — there is no CPU kernel to fall back to."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

OPS = ["layernorm_fwd", "layernorm_bwd", "layernorm_bwd_lp", "layernorm_bwd_add", "layernorm_bwd_scaled_add", "gemm", "gemm_gelu", "gemm_gelu_h", "gemm_residual_lp", "weight_grad", "gemm_tn", "cast", "grad_scale", "row_scale_add", "bn_eval",
       "transpose2d", "weight_refresh", "transpose_batched", "add_readout_cast", "add_readout_amax", "add_readout_cast_scaled", "layernorm_bwd_scaled", "attn_fwd", "attn_fwd_fp8", "attn_bwd", "attn_bwd_fp8", "im2col", "tokens_fwd", "tokens_bwd",
       "pos_interp", "pos_interp_bwd", "row_mean", "score_map", "score_concat", "bilinear", "bilinear_bwd", "bn_fwd", "bn_bwd", "bn_fwd_rows", "bn_bwd_rows",
       "conv3x3", "conv3x3_wgrad", "upsample_ce", "upsample_silog_sums", "upsample_silog_grad", "cityscapes_prepare"]


@pytest.fixture(scope="module")
def D():
    from denseclip_vit_multimodal_amd import _torch_ops
    return _torch_ops.load()


def test_every_op_is_registered(D):
    names = {n for n in torch._C._dispatch_get_all_op_names() if n.startswith("dclip::")}
    assert names == {"dclip::" + o for o in OPS}


def test_fake_shapes_of_the_vit_block_ops(D):
    B, N, H = 2, 129, 12
    C = 64 * H
    with FakeTensorMode():
        x = torch.empty(B * N, C, device="cuda")
        w = torch.empty(C, device="cuda")
        y, mu, rs = D.layernorm_fwd(x, w, w, torch.bfloat16, 1e-5)
        assert y.shape == (B * N, C) and y.dtype == torch.bfloat16 and mu.shape == (B * N,)
        Wqkv = torch.empty(3 * C, C, device="cuda", dtype=torch.bfloat16)
        qkv = D.gemm(y, Wqkv, 5, torch.empty(3 * C, device="cuda"), torch.empty(3 * C, device="cuda"),
                     torch.bfloat16, 1.0)
        assert qkv.shape == (B * N, 3 * C)
        o, lse = D.attn_fwd(qkv, B, N, H, 0.125)
        assert o.shape == (B * N, C) and lse.shape == (B * H * N,) and lse.dtype == torch.float32
        dqkv = D.attn_bwd(qkv, o, o, lse, B, N, H, 0.125)
        assert dqkv.shape == qkv.shape and dqkv.dtype == qkv.dtype
        z, h = D.gemm_gelu(y, torch.empty(4 * C, C, device="cuda", dtype=torch.bfloat16), None)
        assert z.shape == h.shape == (B * N, 4 * C)
        dW = D.weight_grad(h, y, 1.0, torch.zeros(4 * C, device="cuda"))
        assert dW.shape == (4 * C, C) and dW.dtype == torch.float32
        dx, lp = D.layernorm_bwd_lp(y, x, w, mu, rs, x, w, w, torch.bfloat16)
        assert dx.dtype == torch.float32 and lp.dtype == torch.bfloat16
        patches = D.im2col(torch.empty(B, 3, 64, 96, device="cuda"), 14, torch.bfloat16)
        assert patches.shape == (B * 4 * 6, 640)


def test_cpu_tensors_are_refused(D):
    with pytest.raises(NotImplementedError, match="CPU"):
        D.cast(torch.randn(3, 4), torch.bfloat16, 1.0)
    with pytest.raises(NotImplementedError, match="CPU"):
        D.attn_fwd(torch.randn(129, 192).to(torch.bfloat16), 1, 129, 1, 0.125)


def test_fake_tracing_keeps_the_custom_ops(D):
    """make_fx in fake mode (what torch.compile / torch.export run first) traces through the fake
    implementations and keeps the dclip ops as graph nodes."""
    from torch.fx.experimental.proxy_tensor import make_fx

    def f(x, w):
        y, _, _ = D.layernorm_fwd(x, w, w, torch.bfloat16, 1e-5)
        return D.cast(y, torch.float32, 2.0)

    gm = make_fx(f, tracing_mode="fake")(torch.empty(8, 64, device="meta"), torch.empty(64, device="meta"))
    targets = {str(n.target) for n in gm.graph.nodes if n.op == "call_function"}
    assert "dclip.layernorm_fwd.default" in targets and "dclip.cast.default" in targets


def test_fake_layernorm_backward_forms_take_the_abi6_arguments(D):
    """the fake kernels of the four LN backward forms accept the ABI-6 arguments
    (dy_scale, dy_ntok) with non-default values, as ReadoutFn's fast path and the fp16 BlockFn
    pass them, so make_fx / torch.compile of the backward traces."""
    from torch.fx.experimental.proxy_tensor import make_fx
    R, C = 16, 768

    def f(dy, x, w, mu, rs, res, add, sc, dw, db, st):
        a = D.layernorm_bwd(dy, x, w, mu, rs, res, dw, db, sc, 8)
        b, lp = D.layernorm_bwd_lp(dy, x, w, mu, rs, res, dw, db, torch.bfloat16, sc)
        c, lp2, p2 = D.layernorm_bwd_scaled(dy, x, w, mu, rs, res, dw, db, st, 1, 16.0, sc)
        d, lp3, p3 = D.layernorm_bwd_scaled_add(dy, x, w, mu, rs, res, add, sc, 8, dw, db, st, 1, 16.0, sc)
        return a, b, lp, c, lp2, p2, d, lp3, p3

    m = "meta"
    args = (torch.empty(R, C, device=m, dtype=torch.float16), torch.empty(R, C, device=m), torch.empty(C, device=m),
            torch.empty(R, device=m), torch.empty(R, device=m), torch.empty(R, C, device=m),
            torch.empty(R, C, device=m, dtype=torch.float16), torch.empty(4, device=m), torch.empty(C, device=m),
            torch.empty(C, device=m), torch.empty(64, device=m))
    gm = make_fx(f, tracing_mode="fake")(*args)
    targets = {str(n.target) for n in gm.graph.nodes if n.op == "call_function"}
    for op in ("layernorm_bwd", "layernorm_bwd_lp", "layernorm_bwd_scaled", "layernorm_bwd_scaled_add"):
        assert f"dclip.{op}.default" in targets
    with FakeTensorMode():
        fa = [torch.empty(a.shape, dtype=a.dtype, device="cuda") for a in args]
        outs = f(*fa)
    assert outs[0].shape == (R, C) and outs[0].dtype == torch.float32
    assert outs[2].dtype == torch.bfloat16 and outs[4].dtype == torch.float16 and outs[7].dtype == torch.float16
