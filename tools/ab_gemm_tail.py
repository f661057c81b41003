"""A/B of the persistent GEMM's M-tail launch (DCLIP_OPT_GEMM_TAIL 0 / 2 / 1) on the ViT-B/16 token GEMMs
at the bench shape (M = 8 x 8193 = 256k + 8), bf16, with the model's epilogues; options interleaved per
round, medians of per-call HIP-event times (main kernel + tail together).  Under rocprofv3 the
tail kernels' own durations are in the kernel stats.

  python tools/ab_gemm_tail.py [rounds] [option id] [values, comma-separated]   (default: 11 0,2,1)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import _native as Nat  # noqa: E402
from denseclip_vit_multimodal_amd import ops as O  # noqa: E402

M, C = 8 * 8193, 768
bf = torch.bfloat16
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
OPT = int(sys.argv[2]) if len(sys.argv) > 2 else Nat.OPT_GEMM_TAIL
opts = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 2, 1]
torch.manual_seed(0)
dev = "cuda"


def mk(n, k):
    return torch.randn(M, k, device=dev).to(bf), (torch.randn(n, k, device=dev) * k ** -0.5).to(bf), torch.randn(n, device=dev)


cases = []
a, w, b = mk(3 * C, C)
cases.append(("qkv store", lambda a=a, w=w, b=b: O.gemm(a, w, bias=b)))
a, w, b = mk(C, C)
res = torch.randn(M, C, device=dev)
cases.append(("out_proj resid", lambda a=a, w=w, b=b: O.gemm(a, w, Nat.EPI_RESIDUAL, bias=b, aux=res)))
a, w, b = mk(4 * C, C)
cases.append(("c_fc gelu", lambda a=a, w=w, b=b: O.gemm(a, w, Nat.EPI_GELU, bias=b)))
a, w, b = mk(C, 4 * C)
cases.append(("c_proj resid", lambda a=a, w=w, b=b: O.gemm(a, w, Nat.EPI_RESIDUAL, bias=b, aux=res)))
a, w, _ = mk(C, 3 * C)
cases.append(("dX in_proj", lambda a=a, w=w: O.gemm(a, w)))
a, w, _ = mk(C, 4 * C)
cases.append(("dX c_fc", lambda a=a, w=w: O.gemm(a, w)))
a, w, _ = mk(4 * C, C)
z = torch.randn(M, 4 * C, device=dev).to(bf)
cases.append(("dX c_proj gelu'", lambda a=a, w=w: O.gemm(a, w, Nat.EPI_GELU_BWD, aux=z)))
for name, n, k in [("dW in_proj", 3 * C, C), ("dW out_proj", C, C), ("dW c_fc", 4 * C, C), ("dW c_proj", C, 4 * C)]:
    dy = torch.randn(M, n, device=dev).to(bf)
    xx = torch.randn(M, k, device=dev).to(bf)
    dbz = torch.zeros(n, device=dev)
    cases.append((name, lambda dy=dy, xx=xx, dbz=dbz: O.weight_grad(dy, xx, db=dbz.zero_())[0]))


def ev(fn, reps=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


# the arms' outputs bitwise (every option here changes scheduling / launch shape, not arithmetic order,
# except the M tail's K split: compared to fp32 summation order instead)
try:
    for n, fn in cases:
        outs = []
        for o in opts:
            Nat.call("dclip_set_option", OPT, o)
            r = fn()
            outs.append(r[0] if isinstance(r, tuple) else r)
        for o, r in zip(opts[1:], outs[1:]):
            same = torch.equal(r[:-8], outs[0][:-8])
            tail = (r[-8:].float() - outs[0][-8:].float()).abs().max().item()
            print(f"{n:16s} opt{o} vs opt{opts[0]}: rows before the tail bitwise {same}, tail max |d| {tail:.2e}", flush=True)
finally:
    Nat.call("dclip_set_option", OPT, 0)
res_t = {(n, o): [] for n, _ in cases for o in opts}
try:
    for r in range(rounds):
        for n, fn in cases:
            for o in (opts if r % 2 == 0 else opts[::-1]):  # ABBA: no arm always first
                Nat.call("dclip_set_option", OPT, o)
                res_t[(n, o)].append(ev(fn))
finally:
    Nat.call("dclip_set_option", OPT, 0)
tot = {o: 0.0 for o in opts}
for n, _ in cases:
    med = {o: sorted(res_t[(n, o)])[rounds // 2] for o in opts}
    for o in opts:
        tot[o] += med[o]
    print(f"{n:16s} " + "  ".join(f"opt{o} {med[o]:7.1f} us" for o in opts) + f"  {opts[0]}-{opts[1]} {med[opts[0]] - med[opts[1]]:+6.1f} us", flush=True)
print("set    " + "  ".join(f"opt{o} {tot[o]:7.1f} us" for o in opts))
