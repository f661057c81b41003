"""Two ranks on ONE GPU (gloo: RCCL refuses two ranks per device) through the bench's DDP train
step (reference train_denseclip.py:1050-1054).

Default: the tiny model, fused head losses and the graph-replayed frozen text path, three steps;
checks that both ranks end with identical parameters.

--grads: mode F (the ViT trainable: BlockFn's backward, the HIP neck / heads)
at MID_CFG widths, one forward / backward per rank on its own shard; every post-all-reduce
gradient is compared with a single-process run of the same model over the same two shards — each
shard's gradients taken separately (BatchNorm is per rank, no SyncBN, models.py:17-19, as in the
reference) and averaged, which is what DDP's mean all-reduce promises.

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \\
      tools/ddp_gpu_check.py [--grads [--img fp32|bf16]]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def params_identical(params):
    flat = torch.cat([p.detach().float().flatten() for p in params])
    all_ = [torch.zeros_like(flat) for _ in range(dist.get_world_size())]
    dist.all_gather(all_, flat)
    return all(torch.equal(all_[0], a) for a in all_[1:])


def steps_check(dev, rank):
    from helpers import TINY_CFG, CITYSCAPES_CLASSES
    from denseclip_vit_multimodal_amd import DenseCLIP
    from denseclip_vit_multimodal_amd.train import freeze_for_mode, make_optimizer, synth_batch, train_step, wrap_ddp
    torch.manual_seed(0)
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **TINY_CFG).to(dev).train()
    m.fused_head_loss = True
    params = freeze_for_mode(m, "F")
    dm = wrap_ddp(m, dev)
    opt = make_optimizer(params)
    batch = synth_batch(2, 64, 128, dev, rank)
    for _ in range(3):
        loss = train_step(dm, opt, batch)
    assert m._text_graph is not None, "text path was not graph-replayed"
    same = params_identical(params)
    if rank == 0:
        print(f"ddp gloo 2 ranks on one GPU: loss {float(loss):.4f}, parameters identical across ranks: {same}")
    return same


def _mid_model(dev, img_dtype):
    from helpers import MID_CFG, CITYSCAPES_CLASSES, spec_state_dict
    from denseclip_vit_multimodal_amd import DenseCLIP
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **MID_CFG)
    m.load_state_dict(spec_state_dict("mid"))
    m.backbone.compute_dtype = torch.float16 if img_dtype == torch.float32 else img_dtype
    m = m.to(dev).train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()
    m.fused_head_loss = True
    return m


def grads_check(dev, rank, world, img_dtype):
    from denseclip_vit_multimodal_amd.train import freeze_for_mode, gradless_parameter_names, loss_fn, synth_batch, wrap_ddp
    m = _mid_model(dev, img_dtype)
    freeze_for_mode(m, "F")
    dead = set(gradless_parameter_names(m))
    dm = wrap_ddp(m, dev)
    img, seg, depth, mask = synth_batch(2, 128, 256, dev, rank, image_dtype=img_dtype)
    loss_fn(dm(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True), seg, depth, mask).backward()
    g_ddp = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.requires_grad and n not in dead}
    same = params_identical([g_ddp[n] for n in sorted(g_ddp)])
    ok = same
    if rank == 0:
        ref = _mid_model(dev, img_dtype)
        freeze_for_mode(ref, "F")
        acc = {}
        for r in range(world):
            ref.zero_grad(set_to_none=True)
            img, seg, depth, mask = synth_batch(2, 128, 256, dev, r, image_dtype=img_dtype)
            loss_fn(ref(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True), seg, depth, mask).backward()
            for n, p in ref.named_parameters():
                if n in g_ddp:
                    acc[n] = acc.get(n, 0) + p.grad.detach().float() / world
        worst, vit = 0.0, 0
        for n, g in g_ddp.items():
            e = float((g.float() - acc[n]).norm() / acc[n].norm().clamp(min=1e-30))
            worst = max(worst, e)
            vit += n.startswith("backbone.transformer")
        ok = ok and worst < 1e-4 and vit >= 24
        print(f"ddp gloo 2 ranks on one GPU, mode F, {str(img_dtype)[6:]} images: {len(g_ddp)} gradients "
              f"({vit} ViT block tensors), worst rel err vs the single-process shard average {worst:.2e}; "
              f"gradients identical across ranks: {same}; grads check ok: {ok}")
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grads", action="store_true")
    ap.add_argument("--img", choices=["fp32", "bf16"], default="fp32")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if a.grads:
        ok = grads_check(dev, rank, world, torch.float32 if a.img == "fp32" else torch.bfloat16)
    else:
        ok = steps_check(dev, rank)
    flag = torch.tensor([0 if ok else 1])
    dist.all_reduce(flag)
    dist.destroy_process_group()
    if int(flag):
        sys.exit(1)


if __name__ == "__main__":
    main()
