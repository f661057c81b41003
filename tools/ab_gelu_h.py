"""A/B in one process: the frozen-backbone forward's c_fc GEMM writing h only (ops.gemm_gelu_h,
the default) against writing z and h (the training form, z discarded), on the mode-R step and
the inference forward.

  python tools/ab_gelu_h.py [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from denseclip_vit_multimodal_amd import ops  # noqa: E402
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    from denseclip_vit_multimodal_amd.train import synth_batch, make_optimizer
    silog = SILogLoss()
    batch = synth_batch(8, 1024, 2048, dev, 0, image_dtype=torch.bfloat16)
    h_only = ops.gemm_gelu_h

    def z_and_h(A, B, bias=None):
        return ops.gemm(A, B, N.EPI_GELU, bias=bias)[1]

    for mode in ("R", "infer"):
        model = bench.make_model(dev, "R")
        if mode == "infer":
            model.eval()
            opt = None
        else:
            model.train()
            opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
        res = {"h only": [], "z and h": []}
        for rnd in range(3):
            for name, fn in (("z and h", z_and_h), ("h only", h_only)):
                ops.gemm_gelu_h = fn
                dt, _, _ = bench.timed(model, opt, batch, steps, 2, silog, 1)
                res[name].append(dt / steps * 1e3)
        ops.gemm_gelu_h = h_only
        for name, v in res.items():
            print(f"mode {mode:5s} {name:8s} ms/step " + " ".join(f"{x:7.2f}" for x in v) + f"  min {min(v):7.2f}")
        del model, opt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
