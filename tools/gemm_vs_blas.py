"""Our MFMA GEMMs (default tile choice; NT with a bias epilogue) vs torch.mm / addmm (hipBLASLt) on the ViT-B/16 token GEMMs at
the bench shape (M = 8 x 8193), random bf16 data, interleaved rounds.  Forward/dX GEMMs are
"NT" (out = A B^T); weight gradients are "TN" (dW = dY^T X, fp32 out).

  python tools/gemm_vs_blas.py [rounds]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402

M, C = 8 * 8193, 768
bf = torch.bfloat16
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
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


cases = []
for name, n, k in [("qkv", 3 * C, C), ("out_proj", C, C), ("c_fc", 4 * C, C), ("c_proj", C, 4 * C),
                   ("dX in_proj", C, 3 * C), ("dX c_fc", C, 4 * C), ("dX c_proj", 4 * C, C)]:
    a = torch.randn(M, k, device="cuda").to(bf)
    w = (torch.randn(n, k, device="cuda") * k ** -0.5).to(bf)
    b = torch.randn(n, device="cuda")  # every token GEMM of the model carries a bias
    cases.append((f"NT {name:11s} N={n:5d} K={k:5d}", lambda a=a, w=w, b=b: O.gemm(a, w, bias=b),
                  lambda a=a, w=w, b=b: torch.addmm(b.to(bf), a, w.t()), 2.0 * M * n * k))
for name, n, k in [("dX in_proj", C, 3 * C), ("dX out_proj", C, C), ("dX c_fc", C, 4 * C)]:
    # the model's dX GEMMs that feed a LayerNorm backward write fp32 and carry no bias
    a = torch.randn(M, k, device="cuda").to(bf)
    w = (torch.randn(n, k, device="cuda") * k ** -0.5).to(bf)
    cases.append((f"NT {name:11s} N={n:5d} K={k:5d} f32", lambda a=a, w=w: O.gemm(a, w, out_dtype=torch.float32),
                  lambda a=a, w=w: torch.mm(a, w.t(), out_dtype=torch.float32), 2.0 * M * n * k))
for name, n, k in [("in_proj", 3 * C, C), ("out_proj", C, C), ("c_fc", 4 * C, C), ("c_proj", C, 4 * C)]:
    dy = torch.randn(M, n, device="cuda").to(bf)
    x = torch.randn(M, k, device="cuda").to(bf)
    cases.append((f"TN dW {name:8s} N={n:5d} K={k:5d}", lambda dy=dy, x=x: O.weight_grad(dy, x),
                  lambda dy=dy, x=x: torch.mm(dy.t(), x), 2.0 * M * n * k))
res = {c[0]: ([], []) for c in cases}
for r in range(rounds):
    for name, ours, blas, fl in cases:
        res[name][0].append(ev(ours))
        res[name][1].append(ev(blas))
tot_o = tot_b = 0.0
for name, ours, blas, fl in cases:
    o = sorted(res[name][0])[rounds // 2]
    b = sorted(res[name][1])[rounds // 2]
    tot_o += o
    tot_b += b
    print(f"{name}  ours {o:7.3f} ms {fl / o / 1e9:7.1f} TF/s | torch.mm {b:7.3f} ms {fl / b / 1e9:7.1f} TF/s", flush=True)
print(f"total ours {tot_o:.3f} ms, torch.mm {tot_b:.3f} ms")
