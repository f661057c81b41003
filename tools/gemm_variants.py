"""A/B the dclip_gemm tile configurations (DCLIP_OPT_GEMM_TILE) in ONE process on the
ViT-B/16 token GEMMs at the bench shape (M = 8 x 8193), random data, interleaved rounds;
checks each variant against the 128x128 kernel's output.

  python tools/gemm_variants.py [rounds] [tiles...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402

M, C = 8 * 8193, 768
bf = torch.bfloat16
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
tiles = [int(x) for x in sys.argv[2:]] or [1, 2, 3]
torch.manual_seed(0)
x = torch.randn(M, C, device="cuda").to(bf)
h4 = torch.randn(M, 4 * C, device="cuda").to(bf)
q3 = torch.randn(M, 3 * C, device="cuda").to(bf)
res = torch.randn(M, C, device="cuda")
scale3 = torch.ones(3 * C, device="cuda")
cases = []
for name, a, n, k, epi in [("qkv STORE_SCALED", x, 3 * C, C, N.EPI_STORE_SCALED), ("out_proj RESIDUAL", x, C, C, N.EPI_RESIDUAL),
                           ("c_fc GELU", x, 4 * C, C, N.EPI_GELU), ("c_proj RESIDUAL", h4, C, 4 * C, N.EPI_RESIDUAL),
                           ("dz GELU_BWD", x, 4 * C, C, N.EPI_GELU_BWD), ("dX c_fc f32", h4, C, 4 * C, N.EPI_STORE),
                           ("dX in_proj f32", q3, C, 3 * C, N.EPI_STORE), ("dX out_proj bf16", x, C, C, N.EPI_STORE)]:
    w = (torch.randn(n, k, device="cuda") * k ** -0.5).to(bf)
    b = torch.randn(n, device="cuda")
    if epi == N.EPI_RESIDUAL:
        fn = (lambda a=a, w=w, b=b: O.gemm(a, w, N.EPI_RESIDUAL, bias=b, aux=res))
    elif epi == N.EPI_STORE_SCALED:
        fn = (lambda a=a, w=w, b=b: O.gemm(a, w, N.EPI_STORE_SCALED, bias=b, aux=scale3))
    elif epi == N.EPI_GELU:
        fn = (lambda a=a, w=w, b=b: O.gemm(a, w, N.EPI_GELU, bias=b)[1])
    elif epi == N.EPI_GELU_BWD:
        fn = (lambda a=a, w=w: O.gemm(a, w, N.EPI_GELU_BWD, aux=h4))
    elif name.endswith("f32"):
        fn = (lambda a=a, w=w: O.gemm(a, w, out_dtype=torch.float32))
    else:
        fn = (lambda a=a, w=w: O.gemm(a, w))
    cases.append((name, fn, 2.0 * M * n * k))


def ev(fn, reps=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for name, fn, fl in cases:
    N.call("dclip_set_option", N.OPT_GEMM_TILE, 1)
    ref = fn().float()
    for t in tiles:
        N.call("dclip_set_option", N.OPT_GEMM_TILE, t)
        y = fn().float()
        err = float((y - ref).norm() / ref.norm())
        if err > 2e-3:
            print(f"MISMATCH {name} tile {t}: rel err {err:.2e}", flush=True)
times = {(c[0], t): [] for c in cases for t in tiles}
for r in range(rounds):
    for name, fn, fl in cases:
        for t in tiles:
            N.call("dclip_set_option", N.OPT_GEMM_TILE, t)
            times[(name, t)].append(ev(fn))
N.call("dclip_set_option", N.OPT_GEMM_TILE, 0)
for name, fn, fl in cases:
    row = f"{name:20s}"
    for t in tiles:
        ms = sorted(times[(name, t)])[rounds // 2]
        row += f" | tile{t} {ms * 1e3:7.1f} us {fl / ms / 1e9:7.1f} TF/s"
    print(row, flush=True)

# ---- weight gradients (TN): DCLIP_OPT_GEMM_TN_TILE variants (1 128x128, 0 256x256 BK64 x2,
# 2 256x256 BK32 x4, 3 256x256 BK32 x5), checked against the 128x128 kernel
TN_TILES = [int(v) for v in os.environ.get("TN_TILES", "1,0,2,3").split(",")]
tn = []
for name, n, k in [("dW qkv", 3 * C, C), ("dW out_proj", C, C), ("dW c_fc", 4 * C, C), ("dW c_proj", C, 4 * C)]:
    dy = torch.randn(M, n, device="cuda").to(bf)
    xx = torch.randn(M, k, device="cuda").to(bf)
    tn.append((name, (lambda dy=dy, xx=xx: O.weight_grad(dy, xx)[0]), 2.0 * M * n * k))
for name, fn, fl in tn:
    N.call("dclip_set_option", N.OPT_GEMM_TN_TILE, 1)
    ref = fn()
    for t in TN_TILES:
        N.call("dclip_set_option", N.OPT_GEMM_TN_TILE, t)
        y = fn()
        err = float((y - ref).norm() / ref.norm())
        if err > 1e-4:
            print(f"MISMATCH {name} tn {t}: rel err {err:.2e}", flush=True)
tt = {(c[0], t): [] for c in tn for t in TN_TILES}
for r in range(rounds):
    for name, fn, fl in tn:
        for t in TN_TILES:
            N.call("dclip_set_option", N.OPT_GEMM_TN_TILE, t)
            tt[(name, t)].append(ev(fn))
N.call("dclip_set_option", N.OPT_GEMM_TN_TILE, 0)
for name, fn, fl in tn:
    row = f"{name:20s}"
    for t in TN_TILES:
        ms = sorted(tt[(name, t)])[rounds // 2]
        row += f" | tn{t} {ms * 1e3:7.1f} us {fl / ms / 1e9:7.1f} TF/s"
    print(row, flush=True)
