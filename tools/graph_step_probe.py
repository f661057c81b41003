"""The headline train step (mode F, B = 8 @ 1024x2048 bf16) eager vs replayed from one HIP graph
(train.CapturedTrainStep), ABBA rounds in one process on one model and one (capturable) optimizer;
then the two arms' parameters after the same number of steps from the same start are compared.

  python tools/graph_step_probe.py [rounds] [steps] [--fp16]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rounds = int(args[0]) if args else 4
    steps = int(args[1]) if len(args) > 1 else 10
    fp16 = "--fp16" in sys.argv
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    from denseclip_vit_multimodal_amd.train import CapturedTrainStep, make_optimizer, synth_batch, train_step
    dev = torch.device("cuda", 0)
    model = bench.make_model(dev, "F")
    if fp16:
        model.backbone.compute_dtype = torch.float16
    model.train()
    opt = make_optimizer([p for p in model.parameters() if p.requires_grad], capturable=True)
    batch = synth_batch(8, 1024, 2048, dev, 0, image_dtype=torch.float32 if fp16 else torch.bfloat16)
    silog = SILogLoss()
    for _ in range(3):
        train_step(model, opt, batch, silog)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cap = CapturedTrainStep(model, opt, batch, silog)
    torch.cuda.synchronize()
    print(f"capture (3 warm-up steps + the capture) {time.perf_counter() - t0:.2f} s", flush=True)
    arms = {"eager": lambda: train_step(model, opt, batch, silog), "graph": lambda: cap()}
    res = {k: [] for k in arms}
    for r in range(rounds):
        for name in (list(arms) if r % 2 == 0 else list(arms)[::-1]):
            fn = arms[name]
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                loss = fn()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            res[name].append(ms)
            print(f"round {r} {name:6s} {ms:8.2f} ms/step  {8e3 / ms:6.2f} img/s  loss {float(loss):.4f}", flush=True)
    for name, v in res.items():
        s = sorted(v)
        print(f"{name:6s} median {s[len(s) // 2]:8.2f} ms/step  ({', '.join(f'{x:.2f}' for x in v)})")
    # the same two steps from the same state, eager and replayed: parameters must agree
    snap = {n: p.detach().clone() for n, p in model.named_parameters()}
    st = {k: {kk: (vv.clone() if torch.is_tensor(vv) else vv) for kk, vv in v.items()} for k, v in opt.state.items()}
    for _ in range(2):
        train_step(model, opt, batch, silog)
    eager = {n: p.detach().clone() for n, p in model.named_parameters()}
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(snap[n])
        for k, v in st.items():
            for kk, vv in v.items():
                if torch.is_tensor(vv):
                    opt.state[k][kk].copy_(vv)
    from denseclip_vit_multimodal_amd import ops
    ops.refresh_weight_copies([p for g in opt.param_groups for p in g["params"]])  # the restored weights' copies
    for _ in range(2):
        cap()
    torch.cuda.synchronize()
    worst = max(((((p.detach() - eager[n]).abs().max() / (eager[n].abs().max() + 1e-30)).item(), n)
                 for n, p in model.named_parameters()))
    print(f"parameters after 2 eager vs 2 replayed steps from one state: worst rel {worst[0]:.3e} ({worst[1]}) "
          f"(the heads' dropout draws differ between the arms)")


if __name__ == "__main__":
    main()
