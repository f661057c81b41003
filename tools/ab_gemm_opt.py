"""A/B the NT GEMM tile variants (DCLIP_OPT_GEMM_TILE values, or --opt=ID) in ONE process on the ViT-B/16
block's seven NT shapes at the headline batch (65544 token rows), interleaved rounds, with the
epilogues the block uses; every variant is checked against the first (max |difference|).

  python tools/ab_gemm_opt.py [values...]   (default 0 7)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import _native as N  # noqa: E402
from denseclip_vit_multimodal_amd import ops  # noqa: E402

args = sys.argv[1:]
OPT = N.OPT_GEMM_TILE
if args and args[0].startswith("--opt="):  # another option id, e.g. --opt=16 (DCLIP_OPT_GEMM_NT)
    OPT = int(args[0][6:])
    args = args[1:]
vals = [int(v) for v in args] or [0, 7]
M = 8 * 8193
bf = torch.bfloat16
torch.manual_seed(0)
# name: (N, K, epilogue)
shapes = {"qkv": (2304, 768, N.EPI_STORE_SCALED), "out_proj": (768, 768, N.EPI_RESIDUAL),
          "c_fc": (3072, 768, N.EPI_GELU), "c_proj": (768, 3072, N.EPI_RESIDUAL),
          "dX in_proj": (768, 2304, N.EPI_STORE), "dX c_fc": (768, 3072, N.EPI_STORE),
          "dX c_proj": (3072, 768, N.EPI_GELU_BWD)}


def call(n, k, epi, A, B, bias, aux):
    if epi == N.EPI_STORE_SCALED:
        return ops.gemm(A, B, epi, bias=bias, aux=aux)
    if epi == N.EPI_RESIDUAL:
        return ops.gemm(A, B, epi, bias=bias, aux=aux)
    if epi == N.EPI_GELU:
        return ops.gemm(A, B, epi, bias=bias)[1]
    if epi == N.EPI_GELU_BWD:
        return ops.gemm(A, B, epi, aux=aux)
    return ops.gemm(A, B, out_dtype=torch.float32)


def ev(fn, reps=5):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


tot = {v: 0.0 for v in vals}
for name, (n, k, epi) in shapes.items():
    A = torch.randn(M, k, device="cuda").to(bf)
    B = (torch.randn(n, k, device="cuda") * k ** -0.5).to(bf)
    bias = torch.randn(n, device="cuda")
    aux = (torch.rand(n, device="cuda") if epi == N.EPI_STORE_SCALED else
           torch.randn(M, n, device="cuda") if epi == N.EPI_RESIDUAL else
           torch.randn(M, n, device="cuda").to(bf) if epi == N.EPI_GELU_BWD else None)
    outs = []
    for v in vals:
        N.call("dclip_set_option", OPT, v)
        outs.append(call(n, k, epi, A, B, bias, aux).float())
    msg = ", ".join(f"tile {v} max|d| {float((o - outs[0]).abs().max()):.2e}" for v, o in zip(vals[1:], outs[1:]))
    t = {v: [] for v in vals}
    for r in range(5):
        for v in vals:
            N.call("dclip_set_option", OPT, v)
            t[v].append(ev(lambda: call(n, k, epi, A, B, bias, aux)))
    fl = 2.0 * M * n * k
    med = {v: sorted(t[v])[2] for v in vals}
    for v in vals:
        tot[v] += med[v]
    print(f"{name:11s} " + "  ".join(f"tile {v}: {med[v]:.3f} ms {fl / med[v] / 1e9:5.0f} TF/s" for v in vals) + "  | " + msg,
          flush=True)
N.call("dclip_set_option", OPT, 0)
print("total " + "  ".join(f"tile {v}: {tot[v]:.3f} ms" for v in vals))
