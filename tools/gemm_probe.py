"""Run the token GEMMs once each at the bench shape (a short target for rocprofv3 --pmc)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402
from denseclip_vit_multimodal_amd import _native as N  # noqa: E402

if os.environ.get("GEMM_TILE"):
    N.call("dclip_set_option", N.OPT_GEMM_TILE, int(os.environ["GEMM_TILE"]))
M, C = 8 * 8193, 768
bf = torch.bfloat16
x = torch.randn(M, C, device="cuda").to(bf)
h4 = torch.randn(M, 4 * C, device="cuda").to(bf)
w = (torch.randn(4 * C, C, device="cuda") * C ** -0.5).to(bf)
w2 = (torch.randn(C, 4 * C, device="cuda") * (4 * C) ** -0.5).to(bf)
for _ in range(2):
    O.gemm(x, w, out_dtype=torch.bfloat16)          # N=3072 K=768 bf16 store
    O.gemm(h4, w2, out_dtype=torch.float32)         # N=768 K=3072 f32 store
    O.weight_grad(h4, x)                            # TN 3072 x 768 over M
torch.cuda.synchronize()
print("done")
