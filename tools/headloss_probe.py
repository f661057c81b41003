"""Fused upsample + loss kernels at the bench shape (B = 8, 19 x 64 x 128 logits -> 1024 x 2048
labels): HIP-event time of the CE forward + backward and of the two SILog passes.

  python tools/headloss_probe.py [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import ops as O  # noqa: E402


def ev(fn, reps):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = "cuda"
    torch.manual_seed(0)
    B, K, h, w, H, W = 8, 19, 64, 128, 1024, 2048
    lg = (torch.randn(B, K, h, w, device=dev) * 3).bfloat16().requires_grad_(True)
    lab = torch.randint(0, K, (B, H, W), device=dev)
    lab[torch.rand(B, H, W, device=dev) < 0.1] = 255
    pred = (torch.rand(B, 1, h, w, device=dev) * 60 + 1).bfloat16().requires_grad_(True)
    gt = 1 + 79 * torch.rand(B, 1, H, W, device=dev)
    mask = torch.rand(B, 1, H, W, device=dev) >= 0.2

    def ce():
        O.UpsampleCEFn.apply(lg, lab, 255).backward()

    def silog():
        O.UpsampleSILogFn.apply(pred, gt, mask, 0.5, 1e-6).backward()

    print(f"CE fwd+bwd    {ev(ce, reps):8.1f} us", flush=True)
    print(f"SILog fwd+bwd {ev(silog, reps):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
