"""DDP's per-step cost at world size 1 (RCCL), variants of the wrapper, one variant per process:

  python tools/ddp_probe.py {none|allreduce|default|static|keepgrad|nobucketview} [steps]

none: no data parallelism (the headline step); allreduce: train.GradAllReduce (wrap_ddp's default
since round 5); default: torch DDP as wrap_ddp(impl="ddp") builds it; static: DDP with static_graph=True;
keepgrad: default + zero_grad(set_to_none=False) (the gradients stay bucket views between steps);
nobucketview: gradient_as_bucket_view=False.  Prints ms/step and the rocclr copy / fill counts are
visible under rocprofv3.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    variant = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    from denseclip_vit_multimodal_amd import train as T
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    dev = torch.device("cuda", 0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29573")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    model = bench.make_model(dev, "F")
    model.train()
    params = [p for p in model.parameters() if p.requires_grad]
    opt = T.make_optimizer(params)
    if variant != "none":
        dist.init_process_group("nccl")
        if variant == "allreduce":
            model = T.wrap_ddp(model, dev, impl="allreduce")
        elif variant == "hooksonly":  # GradAllReduce's hooks and bookkeeping, no collective calls
            model = T.wrap_ddp(model, dev, impl="allreduce")
            model._launch = lambda i: model._pending["launched"].__setitem__(i, True)
        elif variant == "nohooks":  # GradAllReduce without hooks: one coalesced AVG all-reduce after backward
            model = T.wrap_ddp(model, dev, impl="allreduce")
            for h in model._hooks:
                h.remove()
        elif variant in ("default", "keepgrad"):
            model = T.wrap_ddp(model, dev, impl="ddp")
        else:
            from torch.nn.parallel import DistributedDataParallel as DDP
            ignore = set(T.gradless_parameter_names(model))
            fq = [f"{mn}.{pn}" for mn, mod in model.named_modules() for pn, _ in mod.named_parameters(recurse=False)
                  if (f"{mn}.{pn}" if mn else pn) in ignore]
            DDP._set_params_and_buffers_to_ignore_for_model(model, sorted(ignore | set(fq)))
            model = DDP(model, device_ids=[0], bucket_cap_mb=100, gradient_as_bucket_view=(variant == "static"),
                        find_unused_parameters=False, static_graph=(variant == "static"))
    batch = T.synth_batch(8, 1024, 2048, dev, 0)
    silog = SILogLoss()

    def step():
        img, seg, depth, mask = batch
        out = model(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True)
        loss = T.loss_fn(out, seg, depth, mask, silog)
        opt.zero_grad(set_to_none=(variant != "keepgrad"))
        loss.backward()
        if variant == "nohooks":
            gs = [p.grad for p in model._module_parameters if p.grad is not None]
            with dist._coalescing_manager(async_ops=True) as cm:
                for g in gs:
                    dist.all_reduce(g, op=dist.ReduceOp.AVG)
            cm.wait()
        T.step_unless_nonfinite(opt, loss, check_grads=False)
        return loss

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(f"{variant:13s} {ms:8.2f} ms/step  loss {float(loss):.4f}", flush=True)
    if variant != "none":
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
