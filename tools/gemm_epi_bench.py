"""The ViT block's GEMMs with their real epilogues (as ops.BlockFn issues them) against the same
GEMM with the plain bf16 STORE epilogue, at the bench shape (M = 8 x 8193), interleaved rounds —
isolates what each fused epilogue costs.

  python tools/gemm_epi_bench.py [rounds] [tile,tile,...]   (DCLIP_OPT_GEMM_TILE values, A/B'd)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402

M, C, H = 8 * 8193, 768, 12
bf = torch.bfloat16
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
tiles = [int(t) for t in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
torch.manual_seed(0)


def ev(fn, reps=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def rnd(*s, dt=bf, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(dt)


x32 = torch.randn(M, C, device="cuda")
a768, a3072 = rnd(M, C), rnd(M, 4 * C)
w_in, w_out, w1, w2 = rnd(3 * C, C, scale=0.03), rnd(C, C, scale=0.03), rnd(4 * C, C, scale=0.03), rnd(C, 4 * C, scale=0.02)
b_in, b_out, b1, b2 = (torch.randn(n, device="cuda") * 0.01 for n in (3 * C, C, 4 * C, C))
qs = O.qkv_scale_vector(C, H, "cuda")
z = rnd(M, 4 * C)
w2t = rnd(4 * C, C, scale=0.02)
cases = [
    ("qkv STORE_SCALED", lambda: O.gemm(a768, w_in, N.EPI_STORE_SCALED, bias=b_in, aux=qs), lambda: O.gemm(a768, w_in),
     2.0 * M * 3 * C * C),
    ("out RESIDUAL", lambda: O.gemm(a768, w_out, N.EPI_RESIDUAL, bias=b_out, aux=x32), lambda: O.gemm(a768, w_out),
     2.0 * M * C * C),
    ("c_fc GELU", lambda: O.gemm(a768, w1, N.EPI_GELU, bias=b1), lambda: O.gemm(a768, w1), 2.0 * M * 4 * C * C),
    ("c_proj RESIDUAL", lambda: O.gemm(a3072, w2, N.EPI_RESIDUAL, bias=b2, aux=x32), lambda: O.gemm(a3072, w2),
     2.0 * M * 4 * C * C),
    ("dz GELU_BWD", lambda: O.gemm(a768, w2t, N.EPI_GELU_BWD, aux=z), lambda: O.gemm(a768, w2t), 2.0 * M * 4 * C * C),
    ("dxh2 STORE f32", lambda: O.gemm(a3072, w2, out_dtype=torch.float32), lambda: O.gemm(a3072, w2),
     2.0 * M * 4 * C * C),
]
res = {(c[0], t): ([], []) for c in cases for t in tiles}
for r in range(rounds):
    for name, epi, plain, fl in cases:
        for t in tiles:
            N.call("dclip_set_option", N.OPT_GEMM_TILE, t)
            res[(name, t)][0].append(ev(epi))
            res[(name, t)][1].append(ev(plain))
N.call("dclip_set_option", N.OPT_GEMM_TILE, 0)
for name, epi, plain, fl in cases:
    for t in tiles:
        e = sorted(res[(name, t)][0])[rounds // 2]
        p = sorted(res[(name, t)][1])[rounds // 2]
        print(f"tile {t} {name:18s} epilogue {e:7.3f} ms {fl / e / 1e9:7.1f} TF/s | plain bf16 store {p:7.3f} ms "
              f"{fl / p / 1e9:7.1f} TF/s", flush=True)
