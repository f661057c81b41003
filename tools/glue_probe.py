"""Where the torch-native ("glue") kernels of a train step come from: torch.profiler over two
bench steps (mode F, B = 8 @ 1024x2048), aten ops with their device time, grouped by op and
input shapes, plus the Python frames that issued the fills / copies / adds.

  python tools/glue_probe.py [bf16|fp16] [--steps 2]
"""
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    steps = 2
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    from denseclip_vit_multimodal_amd.train import synth_batch, make_optimizer
    dev = torch.device("cuda", 0)
    model = bench.make_model(dev, "F")
    if dt == "fp16":
        model.backbone.compute_dtype = torch.float16
    model.train()
    opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
    batch = synth_batch(8, 1024, 2048, dev, 0, image_dtype=torch.float32 if dt == "fp16" else torch.bfloat16)
    silog = SILogLoss()
    bench.run_steps(model, opt, batch, 3, silog)
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        bench.run_steps(model, opt, batch, steps, silog)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    rows = []
    for e in ka:
        dev_us = getattr(e, "self_device_time_total", None)
        if dev_us is None:
            dev_us = e.self_cuda_time_total
        if e.key.startswith("aten::") and dev_us > 0:
            rows.append((dev_us / steps, e.count / steps, e.key, str(e.input_shapes)[:110]))
    rows.sort(reverse=True)
    print(f"== {dt}: aten ops with device time, per step (us, calls) ==")
    tot = 0.0
    for us, n, k, shp in rows[:60]:
        print(f"{us:9.1f} {n:6.1f}  {k:28s} {shp}")
    tot = sum(r[0] for r in rows)
    print(f"total aten device time per step: {tot / 1e3:.2f} ms")
    # issuing frames of the glue ops (first frame inside this repo)
    by_src = defaultdict(lambda: [0.0, 0])
    for e in prof.events():
        if not e.name.startswith(("aten::fill_", "aten::zero_", "aten::copy_", "aten::add", "aten::mul",
                                  "aten::zeros", "aten::cat", "aten::where", "aten::_foreach", "aten::clone",
                                  "aten::to", "aten::_to_copy", "aten::stack", "aten::index", "aten::sum")):
            continue
        dev_us = getattr(e, "self_device_time_total", 0) or 0
        kids = sum((getattr(c, "device_time_total", 0) or 0) for c in e.cpu_children)
        us = max(dev_us, getattr(e, "device_time_total", 0) or 0)
        frame = "?"
        for fr in (e.stack or []):
            if "denseclip_vit_multimodal_amd" in fr or "bench.py" in fr or "/torch/optim" in fr:
                frame = fr
                break
        by_src[(e.name, frame)][0] += us / steps
        by_src[(e.name, frame)][1] += 1 / steps
        del kids
    print("== issuing frames (device us per step, calls per step) ==")
    for (name, fr), (us, n) in sorted(by_src.items(), key=lambda kv: -kv[1][0])[:50]:
        if us < 5:
            continue
        print(f"{us:9.1f} {n:6.1f}  {name:22s} {fr}")


if __name__ == "__main__":
    main()
