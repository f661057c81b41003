"""LayerNorm backward at the bench shape (65544 x 768 f32): with and without the dw / db
atomics, with and without the residual and the 16-bit copy — where its time goes.

  python tools/ln_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402
from denseclip_vit_multimodal_amd import ops  # noqa: E402


def main():
    rows, cols = 8 * 8193, 768
    dev = "cuda"
    x = torch.randn(rows, cols, device=dev)
    dy = torch.randn(rows, cols, device=dev)
    res = torch.randn(rows, cols, device=dev)
    w = torch.rand(cols, device=dev) + 0.5
    b = torch.randn(cols, device=dev)
    _, mean, rstd = ops.layernorm_fwd(x, w, b, torch.bfloat16)
    dx = torch.empty_like(x)
    lp = torch.empty(rows, cols, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(cols, device=dev)
    db = torch.zeros(cols, device=dev)
    L = N.lib()
    st = torch.cuda.current_stream().cuda_stream
    P = ops._p

    def call(with_res, with_lp, with_w):
        rc = L.dclip_layernorm_bwd_res(P(dy), N.F32, P(x), N.F32, P(w), P(mean), P(rstd), P(res) if with_res else None,
                                       P(dx), P(lp) if with_lp else None, N.BF16, P(dw) if with_w else None,
                                       P(db) if with_w else None, rows, cols, st)
        assert rc == 0

    def ev(fn, reps=20):
        fn()
        torch.cuda.synchronize()
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return a.elapsed_time(e) / reps * 1e3

    for rnd in range(2):
        for res_, lp_, w_ in ((True, True, True), (True, True, False), (True, False, True), (False, False, True),
                              (False, False, False)):
            us = ev(lambda: call(res_, lp_, w_))
            nbytes = rows * cols * 4 * (3 + (1 if res_ else 0)) + (rows * cols * 2 if lp_ else 0)
            print(f"round {rnd} res {res_:d} lp {lp_:d} dw/db {w_:d}: {us:7.1f} us  {nbytes / us / 1e3:.2f} TB/s",
                  flush=True)
        us = ev(lambda: ops.layernorm_fwd(x, w, b, torch.bfloat16))
        print(f"round {rnd} ln_fwd: {us:7.1f} us  {rows * cols * 6 / us / 1e3:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
