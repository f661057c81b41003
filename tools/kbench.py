"""Kernel micro-benchmarks at the ViT-B/16 1024x2048, batch-8 shapes (M = 8*8193 tokens).

  python tools/kbench.py [--only gemm|attn|misc]

Each op: 3 warm-up launches, then the median of 10 event-timed launches on random data.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402

B, NT, C, H = 8, 8193, 768, 12
M = B * NT
dev = "cuda"
bf = torch.bfloat16


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def report(name, ms, flops=None, bytes_=None):
    s = f"{name:44s} {ms * 1e3:9.1f} us"
    if flops:
        s += f"  {flops / ms / 1e9:8.1f} TF/s ({100 * flops / ms / 1e9 / 2500:.1f}% of 2.5 PF)"
    if bytes_:
        s += f"  {bytes_ / ms / 1e6:8.1f} GB/s"
    print(s, flush=True)


def gemms():
    x = torch.randn(M, C, device=dev).to(bf)
    h4 = torch.randn(M, 4 * C, device=dev).to(bf)
    res = torch.randn(M, C, device=dev)
    for (n, k, epi, a) in [(3 * C, C, N.EPI_STORE, x), (C, C, N.EPI_RESIDUAL, x), (4 * C, C, N.EPI_GELU, x),
                           (C, 4 * C, N.EPI_RESIDUAL, h4)]:
        w = (torch.randn(n, k, device=dev) * k ** -0.5).to(bf)
        bias = torch.randn(n, device=dev)
        aux = res if epi == N.EPI_RESIDUAL else None
        out = res if epi == N.EPI_RESIDUAL else None
        ms = timeit(lambda: O.gemm(a, w, epi, bias=bias, aux=aux, out=out))
        report(f"gemm epi{epi} M={M} N={n} K={k}", ms, 2.0 * M * n * k)
    z = torch.randn(M, 4 * C, device=dev).to(bf)
    dy = torch.randn(M, C, device=dev).to(bf)
    w = torch.randn(4 * C, C, device=dev).to(bf)
    ms = timeit(lambda: O.gemm(dy, w, N.EPI_GELU_BWD, aux=z))
    report(f"gemm gelu_bwd M={M} N={4 * C} K={C}", ms, 2.0 * M * 4 * C * C)
    w2 = torch.randn(C, 4 * C, device=dev).to(bf)
    ms = timeit(lambda: O.gemm(z, w2, out_dtype=torch.float32))
    report(f"gemm dX f32 M={M} N={C} K={4 * C}", ms, 2.0 * M * 4 * C * C)
    for (n, k, a, b) in [(4 * C, C, z, x), (C, 4 * C, dy, h4), (3 * C, C, torch.randn(M, 3 * C, device=dev).to(bf), x)]:
        ms = timeit(lambda: O.weight_grad(a, b))
        report(f"weight_grad N={n} K={k} (M={M})", ms, 2.0 * M * n * k)
    ms = timeit(lambda: O.transpose(h4, M, 4 * C, bf, rows_pad=M + 56))
    report("transpose M x 3072 bf16", ms, None, 2 * M * 4 * C * 2)


def attn():
    qkv = torch.randn(M, 3 * C, device=dev).to(bf)
    dout = torch.randn(M, C, device=dev).to(bf)
    fl = 4.0 * B * H * NT * NT * 64
    ms = timeit(lambda: O.attn_fwd(qkv, B, NT, H, 0.125))
    report("attn_fwd", ms, fl)
    ms = timeit(lambda: O.attn_fwd_fp8(qkv, B, NT, H))
    report("attn_fwd_fp8 (row 0 + pack + e4m3 MX kernel)", ms, fl)
    o, lse = O.attn_fwd(qkv, B, NT, H, 0.125)
    ms = timeit(lambda: O.attn_bwd(qkv, o, dout, lse, B, NT, H, 0.125))
    report("attn_bwd (delta+dq+dkdv), 2.5x fwd flops", ms, 2.5 * fl)


def misc():
    x = torch.randn(M, C, device=dev)
    w = torch.randn(C, device=dev)
    b = torch.randn(C, device=dev)
    ms = timeit(lambda: O.layernorm_fwd(x, w, b, bf))
    report("layernorm_fwd f32->bf16", ms, None, M * C * 6)
    _, mu, rs = O.layernorm_fwd(x, w, b, bf)
    dy = torch.randn(M, C, device=dev)
    dx = torch.empty_like(x)
    dw = torch.zeros(C, device=dev)
    ms = timeit(lambda: O.layernorm_bwd(dy, x, w, mu, rs, dx, 1, dw, dw))
    report("layernorm_bwd f32 (accumulate)", ms, None, M * C * 16)
    ms = timeit(lambda: O.cast(x, bf))
    report("cast f32->bf16", ms, None, M * C * 6)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="all")
    a = ap.parse_args()
    for name, fn in (("gemm", gemms), ("attn", attn), ("misc", misc)):
        if a.only in ("all", name):
            fn()
