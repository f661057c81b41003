"""Time the attention forward at the bench shape (B 8, N 8193, 12 heads): the bf16 kernel and
dclip_attn_fwd_fp8 in both modes (default: 16-bit scores + fp8 P V; DCLIP_OPT_ATTN_FP8_QK 1:
all e4m3), alternated in one process.  Run under rocprofv3 --kernel-trace --stats to split the
pack / row-0 / main kernels.

  python tools/fp8_modes_probe.py [reps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from denseclip_vit_multimodal_amd import _native as NATIVE  # noqa: E402
from denseclip_vit_multimodal_amd import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    B, N, H = 8, 8193, 12
    C = 64 * H
    torch.manual_seed(0)
    qkv = (torch.randn(B * N, 3 * C, device="cuda") * 1.5).to(torch.bfloat16)
    qkv[:, :C] = (qkv[:, :C].float() * (64 ** -0.5 * 1.4426950408889634)).to(torch.bfloat16)
    lib = NATIVE.lib()
    fl = 4.0 * B * H * N * N * 64

    def ev(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    for rnd in range(2):
        t16 = ev(lambda: ops.attn_fwd(qkv, B, N, H, 64 ** -0.5))
        lib.dclip_set_option(NATIVE.OPT_ATTN_FP8_QK, 0)
        ts = ev(lambda: ops.attn_fwd_fp8(qkv, B, N, H))
        lib.dclip_set_option(NATIVE.OPT_ATTN_FP8_QK, 1)
        tq = ev(lambda: ops.attn_fwd_fp8(qkv, B, N, H))
        lib.dclip_set_option(NATIVE.OPT_ATTN_FP8_QK, 0)
        print(f"round {rnd}: bf16 {t16:.4f} ms ({fl / t16 / 1e9:.0f} TF/s) | fp8 S16 {ts:.4f} ms "
              f"({fl / ts / 1e9:.0f}) | fp8 all-e4m3 {tq:.4f} ms ({fl / tq / 1e9:.0f})", flush=True)


if __name__ == "__main__":
    main()
