"""Subprocess body of test_gpu_headline.test_grad_allreduce_rccl_world_size_1 (its own process, so
the RCCL process group it creates does not outlive it).

One rank on an RCCL ("nccl") group: the ViT-B/16 mode-F DenseCLIP of the benchmark (every op on the
HIP kernels, the fused resize + losses) in bf16 at 2 x 128 x 256, trained one step bare and one
step under train.GradAllReduce with the collectives issued (skip_collectives False: at world size 1
the wrapper otherwise skips the identity), coalesced and per-tensor, ~1 MB buckets.  The AVG
all-reduce of one rank is x / 1 and the step is bitwise reproducible since ABI 7 (fixed-order loss
folds, tests/test_gpu_determinism.py), so every gradient must come back BIT-IDENTICAL to the bare
model's (a collective that read a gradient before its producer wrote it would not); every bucket
must have been launched, in bucket order.  Prints one JSON line."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402


def make():
    import bench
    torch.manual_seed(0)
    m = bench.make_model(torch.device("cuda"), "F").train()
    m.backbone.compute_dtype = torch.bfloat16
    for mod in m.modules():
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    return m


def grads(model, batch):
    from denseclip_vit_multimodal_amd.train import loss_fn
    img, seg, depth, mask = batch
    out = model(img, gt_semantic_seg=seg, gt_depth=depth, return_loss=True)
    loss = loss_fn(out, seg, depth, mask)
    loss.backward()
    torch.cuda.synchronize()
    inner = model.module if hasattr(model, "module") else model
    return {n: p.grad.detach().clone() for n, p in inner.named_parameters() if p.grad is not None}


def main():
    from denseclip_vit_multimodal_amd.train import GradAllReduce, synth_batch
    dist.init_process_group("nccl")
    try:
        batch = synth_batch(2, 128, 256, torch.device("cuda"), 0, image_dtype=torch.bfloat16)
        ref = grads(make(), batch)
        res = {"grads": len(ref)}
        for coalesce in (True, False):
            w = GradAllReduce(make(), bucket_cap_mb=1, last_bucket_cap_mb=1)
            w.skip_collectives = False
            w.coalesce = coalesce
            launched = []
            orig = w._launch

            def count(i, orig=orig, launched=launched):
                launched.append(i)
                orig(i)

            w._launch = count
            g = grads(w, batch)
            assert set(g) == set(ref), sorted(set(g) ^ set(ref))
            bad = [n for n in ref if not torch.equal(g[n], ref[n])]
            assert not bad, (len(bad), bad[:5])
            assert launched == list(range(len(w._buckets))), (launched, len(w._buckets))
            res[f"buckets_coalesce_{coalesce}"] = len(w._buckets)
        # the tile walk under collectives: CUs held by a side-stream occupier
        # (tools/cu_hog.hip, standing in for RCCL's channel kernels, which at world size 1 launch
        # nothing) from every bucket launch, the GEMMs of the rest of the backward on the claims
        # walk — the gradients still bit-identical, the walk back to static after the backward
        import ctypes
        from denseclip_vit_multimodal_amd import ops
        hog = ctypes.CDLL(os.path.join(os.path.dirname(HERE), "tools", "libcu_hog.so"))
        hog.cu_hog.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
        sink = torch.zeros(64, dtype=torch.int32, device="cuda")
        side = torch.cuda.Stream()
        w = GradAllReduce(make(), bucket_cap_mb=25, last_bucket_cap_mb=25)
        w.skip_collectives = False
        assert w.gemm_walk_under_collectives == 1
        orig = w._launch
        walks = []

        def hog_launch(i, orig=orig):
            side.wait_stream(torch.cuda.current_stream())
            assert hog.cu_hog(16, 300.0, sink.data_ptr(), side.cuda_stream) == 0
            orig(i)
            walks.append(ops._GEMM_WALK[0])

        w._launch = hog_launch
        g = grads(w, batch)
        torch.cuda.synchronize()
        bad = [n for n in ref if not torch.equal(g[n], ref[n])]
        assert not bad, (len(bad), bad[:5])
        assert walks and all(x == 1 for x in walks), walks
        assert ops._GEMM_WALK[0] == 0
        res["hog_windows"] = len(walks)
        print(json.dumps(res))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
