"""torch.ops.dclip.* on the GPU: torch.library.opcheck (schema / mutation annotations, fake vs
real shapes and strides, AOT dispatch with dynamic shapes) on the ViT block's ops, and a whole
ViT block (forward and backward) captured in a HIP graph with torch.cuda.graph and replayed."""
import pytest
import torch

from helpers import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _need(hip):
    torch.manual_seed(0)


def D():
    from denseclip_vit_multimodal_amd import ops
    return ops.D()


def _opcheck(op, args):
    torch.library.opcheck(op, args, test_utils=("test_schema", "test_faketensor", "test_aot_dispatch_dynamic"))


def test_opcheck_layernorm():
    x = torch.randn(300, 768, device=DEV)
    w = torch.randn(768, device=DEV)
    b = torch.randn(768, device=DEV)
    _opcheck(D().layernorm_fwd, (x, w, b, torch.bfloat16, 1e-5))
    _, mu, rs = D().layernorm_fwd(x, w, b, torch.float32, 1e-5)
    dy = torch.randn(300, 768, device=DEV).to(torch.bfloat16)
    _opcheck(D().layernorm_bwd, (dy, x, w, mu, rs, None, torch.zeros(768, device=DEV), torch.zeros(768, device=DEV)))
    _opcheck(D().layernorm_bwd_lp, (dy, x, w, mu, rs, x.clone(), torch.zeros(768, device=DEV),
                                    torch.zeros(768, device=DEV), torch.bfloat16))
    # ABI 6 arguments with non-default values (the fake kernels must take them)
    sc = torch.tensor([4.0, 0.25, 0.0, 0.0], device=DEV)
    dyh = (torch.randn(300, 768, device=DEV) * 4).to(torch.float16)
    _opcheck(D().layernorm_bwd, (dyh, x, w, mu, rs, None, torch.zeros(768, device=DEV), torch.zeros(768, device=DEV),
                                 sc, 100))
    _opcheck(D().layernorm_bwd_lp, (dyh, x, w, mu, rs, x.clone(), torch.zeros(768, device=DEV),
                                    torch.zeros(768, device=DEV), torch.bfloat16, sc))


def test_opcheck_gemm_family():
    A = torch.randn(520, 768, device=DEV).to(torch.bfloat16)
    B = torch.randn(256, 768, device=DEV).to(torch.bfloat16)
    bias = torch.randn(256, device=DEV)
    _opcheck(D().gemm, (A, B, 0, bias, None, torch.float32, 1.0))
    _opcheck(D().gemm, (A, B, 2, bias, torch.randn(520, 256, device=DEV), torch.float32, 1.0))
    _opcheck(D().gemm_gelu, (A, B, bias))
    dy = torch.randn(520, 256, device=DEV).to(torch.bfloat16)
    _opcheck(D().weight_grad, (dy, A, 1.0, torch.zeros(256, device=DEV)))
    _opcheck(D().cast, (torch.randn(77, 64, device=DEV), torch.bfloat16, 4.0))
    _opcheck(D().transpose2d, (torch.randn(72, 136, device=DEV), torch.bfloat16))


def test_opcheck_attention():
    from test_gpu_kernels import prescale
    B, N, H = 2, 257, 2
    qkv, _ = prescale(torch.randn(B * N, 3 * 64 * H, device=DEV).to(torch.bfloat16), H)
    _opcheck(D().attn_fwd, (qkv, B, N, H, 0.125))
    o, lse = D().attn_fwd(qkv, B, N, H, 0.125)
    _opcheck(D().attn_bwd, (qkv, o, torch.randn_like(o), lse, B, N, H, 0.125))
    _opcheck(D().attn_fwd_fp8, (qkv, B, N, H))


def test_opcheck_resize_and_bn():
    x = torch.randn(2, 19, 8, 16, device=DEV)
    _opcheck(D().bilinear, (x, 64, 128, torch.float32))
    _opcheck(D().bilinear_bwd, (torch.randn(2, 19, 64, 128, device=DEV), 8, 16))
    m = torch.randn(2, 128, 6, 10, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    _opcheck(D().bn_fwd, (m, torch.rand(128, device=DEV), torch.randn(128, device=DEV), torch.zeros(128, device=DEV),
                          torch.ones(128, device=DEV), 0.1, 1e-5, True))
    buf = torch.randn(300, 1536, device=DEV).to(torch.bfloat16)
    _opcheck(D().bn_fwd_rows, (buf[:, 128:256], torch.rand(128, device=DEV), torch.randn(128, device=DEV), None, None,
                               0.1, 1e-5, True, torch.empty(300, 1536, device=DEV, dtype=torch.bfloat16)[:, 128:256]))
    _opcheck(D().bn_eval, (m, torch.rand(128, device=DEV), torch.randn(128, device=DEV), torch.randn(128, device=DEV),
                           torch.rand(128, device=DEV) + 0.5, 1e-5, True))
    g = torch.randn(4096, device=DEV) * 1e-7
    _opcheck(D().grad_scale, (g, 16.0))
    _opcheck(D().row_scale_add, (torch.randn(258, 64, device=DEV), torch.randn(258, 64, device=DEV),
                                 torch.rand(129, device=DEV)))


def _block(C=768, H=12):
    from denseclip_vit_multimodal_amd.models import ResidualAttentionBlock
    blk = ResidualAttentionBlock(C, H).to(DEV)
    with torch.no_grad():
        for p in blk.parameters():
            if p.dim() > 1:
                p.normal_(0, C ** -0.5)
            else:
                p.normal_(0, 0.1)
    return blk


def test_vit_block_hip_graph_capture_fwd_bwd():
    """One ViT-B block (B = 2, N = 1025, bf16 operands) forward + backward captured with
    torch.cuda.graph: the replay reproduces the eager output and every gradient bit for bit (the
    ops are stream-ordered, never synchronise with the host, and since ABI 5 the LayerNorm dw / db
    come from a per-call partials table summed in a fixed order instead of float atomics)."""
    from denseclip_vit_multimodal_amd import ops
    blk = _block()
    B, N, H, C = 2, 1025, 12, 768
    meta = (B, N, H, torch.bfloat16, False)
    x = torch.randn(B * N, C, device=DEV).requires_grad_(True)
    gy = torch.randn(B * N, C, device=DEV)

    def step():
        y = ops.BlockFn.apply(x, meta, *blk.hip_params())
        y.backward(gy)
        return y

    # eager reference (and warm-up: allocator, cached weight casts) on a side stream
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            x.grad = None
            blk.zero_grad(set_to_none=True)
            y_ref = step().detach().clone()
    torch.cuda.current_stream().wait_stream(s)
    gx_ref = x.grad.clone()
    gw_ref = {n: p.grad.clone() for n, p in blk.named_parameters() if p.grad is not None}
    x.grad = None
    blk.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y_static = step()
    for _ in range(2):  # grads are graph outputs (re-written, not accumulated, by each replay)
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y_static, y_ref)
    assert torch.equal(x.grad, gx_ref)
    assert len(gw_ref) == 12
    for n, p in blk.named_parameters():
        assert torch.equal(p.grad, gw_ref[n]), (n, rel_err(p.grad, gw_ref[n]))


def test_custom_ops_reject_bad_dtypes_and_sizes():
    """the ops check the f32 vectors and side inputs the kernels index by the GEMM / BN
    widths — a half-precision bias, a mis-sized aux or db, mismatched weight-gradient operands or
    16-bit running statistics raise instead of reading or writing past a buffer."""
    bf = torch.bfloat16
    A = torch.randn(256, 128, device=DEV).to(bf)
    B = torch.randn(64, 128, device=DEV).to(bf)
    good = torch.randn(64, device=DEV)
    with pytest.raises(RuntimeError, match="float32"):
        D().gemm(A, B, 0, good.half(), None, bf, 1.0)
    with pytest.raises(RuntimeError, match="elements"):
        D().gemm(A, B, 0, torch.randn(63, device=DEV), None, bf, 1.0)
    with pytest.raises(RuntimeError, match=r"\(M, N\)"):
        D().gemm(A, B, 2, good, torch.randn(256, 32, device=DEV), torch.float32, 1.0)
    with pytest.raises(RuntimeError, match=r"\(M, N\)"):
        D().gemm(A, B, 3, None, None, bf, 1.0)
    with pytest.raises(RuntimeError, match="scale"):
        D().gemm(A, B, 5, good, torch.randn(32, device=DEV), bf, 1.0)
    with pytest.raises(RuntimeError, match="elements"):
        D().gemm_gelu(A, B, torch.randn(65, device=DEV))
    dy = torch.randn(256, 64, device=DEV)
    with pytest.raises(RuntimeError, match="dtypes differ"):
        D().weight_grad(dy.half(), A, 1.0, torch.zeros(64, device=DEV))
    with pytest.raises(RuntimeError, match="elements"):
        D().weight_grad(dy.to(bf), A, 1.0, torch.zeros(32, device=DEV))
    x = torch.randn(2, 64, 4, 4, device=DEV).to(bf).contiguous(memory_format=torch.channels_last)
    w, b = torch.ones(64, device=DEV), torch.zeros(64, device=DEV)
    with pytest.raises(RuntimeError, match="float32"):
        D().bn_eval(x, w, b, torch.zeros(64, device=DEV).half(), torch.ones(64, device=DEV), 1e-5, False)
    with pytest.raises(RuntimeError, match="elements"):
        D().bn_fwd(x, w[:32], b, None, None, 0.1, 1e-5, False)
    with pytest.raises(RuntimeError, match="elements"):
        D().layernorm_fwd(torch.randn(8, 64, device=DEV), w[:32], b, torch.float32, 1e-5)
    # and the good calls still run
    D().gemm(A, B, 0, good, None, bf, 1.0)
    D().bn_eval(x, w, b, torch.zeros(64, device=DEV), torch.ones(64, device=DEV), 1e-5, True)


@pytest.mark.parametrize("M", [520, 65544])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_gemm_residual_lp_copy(M, dt):
    """The residual epilogue's 16-bit copy (the read-out map's token buffer, BlockFn): the f32
    output equals the plain residual GEMM and the copy equals its cast, bit for bit — both the
    persistent kernel's epilogue and the row-tail path (M = 8 x 8193 = 65544 rows)."""
    A = torch.randn(M, 768, device=DEV).to(dt)
    B = torch.randn(256, 768, device=DEV).to(dt)
    bias = torch.randn(256, device=DEV)
    aux = torch.randn(M, 256, device=DEV)
    out, lp = D().gemm_residual_lp(A, B, bias, aux)
    ref = D().gemm(A, B, 2, bias, aux, torch.float32, 1.0)
    assert torch.equal(out, ref)
    assert lp.dtype == dt and torch.equal(lp, ref.to(dt))
    if M == 520:
        _opcheck(D().gemm_residual_lp, (A, B, bias, aux))
