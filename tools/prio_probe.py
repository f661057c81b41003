"""Does a high-priority main stream shorten the step (the text graph then replays on a queue of
lower priority than the backbone's)?  Mode F, B = 8 @ 1024x2048 bf16, arms alternating in one
process: the default stream vs a stream of the highest priority torch offers.

  python tools/prio_probe.py [rounds] [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    from denseclip_vit_multimodal_amd.train import synth_batch, make_optimizer
    dev = torch.device("cuda", 0)
    lo, hi = torch.cuda.Stream.priority_range()
    print(f"stream priority range: low {lo}, high {hi}", flush=True)
    model = bench.make_model(dev, "F")
    model.train()
    opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
    batch = synth_batch(8, 1024, 2048, dev, 0, image_dtype=torch.bfloat16)
    silog = SILogLoss()
    fast = torch.cuda.Stream(device=dev, priority=hi)
    res = {"default": [], "high-priority main": []}
    for r in range(rounds):
        for name in res:
            s = torch.cuda.current_stream(dev) if name == "default" else fast
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                bench.run_steps(model, opt, batch, 3, silog)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                bench.run_steps(model, opt, batch, steps, silog)
                torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            res[name].append(ms)
            print(f"round {r} {name:20s} {ms:8.2f} ms/step", flush=True)
    for k, v in res.items():
        sv = sorted(v)
        print(f"{k:20s} median {sv[len(sv) // 2]:8.2f} ms/step ({', '.join(f'{x:.2f}' for x in v)})")


if __name__ == "__main__":
    main()
