"""A/B of the persistent GEMMs' tile walk under injected collective windows.

One process, one rank on an RCCL group (world size 1), the benchmark's ViT-B/16 mode-F step under
train.GradAllReduce with the collectives issued.  At world size 1 RCCL's all-reduce launches no
kernel, so the CUs its channel kernels would hold on an 8-GPU node are emulated: every bucket
launch also starts tools/cu_hog.hip on a side stream (after the bucket's gradients are ready, as
RCCL's kernels would), holding `--held` CUs for `--usec` microseconds (one-wave workgroups with
96 KiB of LDS: no GEMM workgroup fits beside one).

Arms, in rotating (ABBA-style) order per round, `--steps` timed steps each:
  plain        no hog, static walk throughout (the uncontended step)
  claims       no hog, the claims walk during the backward (what N > 1 runs when the CUs are free)
  hog_static   hog windows, static walk (round 5's behaviour)
  hog_claims   hog windows, the claims walk between the first bucket's launch and the end of the
               backward (GradAllReduce.gemm_walk_under_collectives = 1, the default)
Then the gradients of one step from the same state under every arm, compared bit for bit.

  python tools/ab_collective_walk.py [--batch 8 --height 1024 --width 2048 --held 16 --usec 600]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--width", type=int, default=2048)
    ap.add_argument("--held", type=int, default=16)
    ap.add_argument("--usec", type=float, default=600.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29581")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    import bench
    from denseclip_vit_multimodal_amd import ops
    from denseclip_vit_multimodal_amd.train import GradAllReduce, loss_fn, make_optimizer, synth_batch, train_step
    dist.init_process_group("nccl")
    dev = torch.device("cuda", 0)
    hog = ctypes.CDLL(os.path.join(ROOT, "tools", "libcu_hog.so"))
    hog.cu_hog.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(device=dev)
    torch.manual_seed(0)
    m = bench.make_model(dev, "F").train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    w = GradAllReduce(m)
    w.skip_collectives = False
    opt = make_optimizer([p for p in m.parameters() if p.requires_grad])
    batch = synth_batch(a.batch, a.height, a.width, dev, 0, image_dtype=torch.bfloat16)
    orig = w._launch
    state = {"hog": False, "windows": 0}

    def launch(i):
        if state["hog"]:  # the emulated channel kernels start when the bucket's gradients are ready
            side.wait_stream(torch.cuda.current_stream(dev))
            assert hog.cu_hog(a.held, a.usec, sink.data_ptr(), side.cuda_stream) == 0
            state["windows"] += 1
        orig(i)

    w._launch = launch

    def arm(name):
        state["hog"] = name.startswith("hog")
        w.gemm_walk_under_collectives = 1 if name.endswith("claims") else None

    arms = ["plain", "claims", "hog_static", "hog_claims"]
    for name in arms:  # warm every path
        arm(name)
        train_step(w, opt, batch)
    torch.cuda.synchronize()
    times = {n: [] for n in arms}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        order = arms[r % 4:] + arms[:r % 4]
        if r % 2:
            order = order[::-1]
        for name in order:
            arm(name)
            state["windows"] = 0
            e0.record()
            for _ in range(a.steps):
                train_step(w, opt, batch)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.steps)
            print(f"round {r} {name:11s} {times[name][-1]:8.2f} ms/step  hog windows {state['windows']}", flush=True)
    mean = {n: sum(v) / len(v) for n, v in times.items()}
    # bitwise: one backward from the same parameters under every arm
    grads = {}
    for name in arms:
        arm(name)
        img, seg, depth, mask = batch
        out = w(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True)
        loss = loss_fn(out, seg, depth, mask)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        torch.cuda.synchronize()
        grads[name] = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    ref = grads["plain"]
    bitwise = {n: all(torch.equal(g[k], ref[k]) for k in ref) for n, g in grads.items()}
    held_share = a.held / torch.cuda.get_device_properties(dev).multi_processor_count
    res = {"ms_per_step": {n: round(v, 3) for n, v in mean.items()},
           "slowdown_vs_plain": {n: round(mean[n] / mean["plain"] - 1, 4) for n in arms},
           "held_cu_share": round(held_share, 4), "hog_usec": a.usec, "buckets": len(w._buckets),
           "grads_bitwise_equal_to_plain": bitwise,
           "config": {"batch": a.batch, "height": a.height, "width": a.width, "steps": a.steps, "rounds": a.rounds}}
    print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
