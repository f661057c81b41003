"""Two ranks on ONE GPU (gloo: RCCL refuses two ranks per device) through the bench's DDP
train step with the tiny model, fused head losses and the graph-replayed frozen text path;
checks that both ranks end with identical parameters.

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \\
      tools/ddp_gpu_check.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
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
    flat = torch.cat([p.detach().float().flatten() for p in params])
    all_ = [torch.zeros_like(flat) for _ in range(2)]
    dist.all_gather(all_, flat)
    same = torch.equal(all_[0], all_[1])
    if rank == 0:
        print(f"ddp gloo 2 ranks on one GPU: loss {float(loss):.4f}, parameters identical across ranks: {same}")
    dist.destroy_process_group()
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
