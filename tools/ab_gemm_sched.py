"""A/B of the NT GEMM's tile walks in ONE process: the persistent kernel's static walk (default), its
work-conserving claims (DCLIP_OPT_GEMM_SCHED 1) and the one-tile-per-workgroup grid kernel
(DCLIP_OPT_GEMM_TILE 2, scheduled by the hardware dispatcher),
with and without CUs held by side-stream kernels (RCCL's channel
kernels, or the text graph's side stream, displace workgroups of a persistent kernel).

  python tools/ab_gemm_sched.py [--rounds 5]

The seven NT GEMM shapes of a ViT-B/16 block at the headline batch (M = 8 * 8193 rows, bf16): the
forward in_proj / out_proj / c_fc / c_proj and the three dX GEMMs, as bare bf16 GEMMs.  "Held" CUs:
tools/cu_hog.hip (tools/libcu_hog.so) on a side stream — `held` one-wave workgroups with 96 KiB of
LDS each, so no GEMM workgroup (160 KiB) fits on their CUs — for about the GEMM set's duration,
launched just before it.  Prints the 7-GEMM set's time per arm and the slowdown against the
uncontended static set; outputs are compared bit for bit across arms.
"""
import ctypes
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from denseclip_vit_multimodal_amd import ops, _native as N  # noqa: E402

SHAPES = [("qkv", 768, 2304), ("out_proj", 768, 768), ("c_fc", 768, 3072), ("c_proj", 3072, 768),
          ("dX in_proj", 2304, 768), ("dX c_fc", 3072, 768), ("dX c_proj", 768, 3072)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--rows", type=int, default=8 * 8193)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    ops_in = []
    for name, k, n in SHAPES:
        A = (torch.randn(a.rows, k, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        B = (torch.randn(n, k, device=dev, generator=g) * k ** -0.5).to(torch.bfloat16)
        ops_in.append((name, A, B))
    lib = N.load()

    def run_set():
        return [ops.gemm(A, B) for _, A, B in ops_in]

    # the set's uncontended duration, to size the sleepers
    for _ in range(3):
        run_set()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run_set()
    e1.record()
    torch.cuda.synchronize()
    set_ms = e0.elapsed_time(e1)
    hog = ctypes.CDLL(os.path.join(ROOT, "tools", "libcu_hog.so"))
    hog.cu_hog.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream()
    usec = set_ms * 1e3 * 1.2
    print(f"uncontended static set {set_ms:.3f} ms; CUs held {usec:.0f} us")
    ref = [o.clone() for o in run_set()]
    res = {}
    for r in range(a.rounds):
        for held in (0, 16, 32):
            for sched in ("static", "claims", "grid"):
                lib.dclip_set_option(N.OPT_GEMM_SCHED, 1 if sched == "claims" else 0)
                lib.dclip_set_option(N.OPT_GEMM_TILE, 2 if sched == "grid" else 0)
                run_set()  # warm (per-stream counters, caches)
                torch.cuda.synchronize()
                if held:
                    assert hog.cu_hog(held, usec, sink.data_ptr(), side.cuda_stream) == 0
                e0.record()
                outs = run_set()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((held, sched), []).append(e0.elapsed_time(e1))
                for o, rf in zip(outs, ref):
                    if sched == "grid":  # another kernel (its own summation order within a tile)
                        assert float((o.float() - rf.float()).norm() / rf.float().norm()) < 1e-2
                    else:
                        assert torch.equal(o, rf), "outputs differ between the tile walks"
    lib.dclip_set_option(N.OPT_GEMM_SCHED, 0)
    lib.dclip_set_option(N.OPT_GEMM_TILE, 0)
    base = sorted(res[(0, "static")])[len(res[(0, "static")]) // 2]
    print(f"{'held CUs':>9} {'walk':>8} {'median ms':>10} {'min ms':>8} {'vs uncontended static':>22}  share held")
    for (held, sched), v in sorted(res.items()):
        v = sorted(v)
        med = v[len(v) // 2]
        print(f"{held:9d} {sched:>8} {med:10.3f} {v[0]:8.3f} {med / base - 1:21.1%}  "
              f"{held / torch.cuda.get_device_properties(0).multi_processor_count:.1%}")
    print("persistent outputs bitwise equal across walks and contention: True")


if __name__ == "__main__":
    main()
