"""A/B two builds of libdclip.so on the attention kernels in ONE process (interleaved rounds,
same device, same random data) — the way to compare code changes (guide §5.4 rule 24).

  python tools/ab_attn.py [-r ROUNDS] [--fp16] libA.so libB.so [libC.so ...]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import _native  # noqa: E402

B, NT, C, H = 8, 8193, 768, 12
args = sys.argv[1:]
rounds = 7
if args[0] == "-r":
    rounds = int(args[1])
    args = args[2:]
DT, TDT = 2, torch.bfloat16
if args[0] == "--fp16":
    DT, TDT = 1, torch.float16
    args = args[1:]
names = args
libs = [_native.load(p) for p in names]
torch.manual_seed(0)
qkv = torch.randn(B * NT, 3 * C, device="cuda").to(TDT)
dout = torch.randn(B * NT, C, device="cuda").to(TDT)
o = torch.empty(B * NT, C, device="cuda", dtype=TDT)
lse = torch.empty(B * H * NT, device="cuda")
delta = torch.empty(libs[0].dclip_attn_bwd_workspace(B, NT, H), device="cuda")
dqkv = torch.empty_like(qkv)
st = torch.cuda.current_stream().cuda_stream


def fwd(L):
    assert L.dclip_attn_fwd(DT, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, NT, H, 64, 0.125, st) == 0


def bwd(L):
    assert L.dclip_attn_bwd(DT, qkv.data_ptr(), o.data_ptr(), dout.data_ptr(), lse.data_ptr(), delta.data_ptr(),
                            dqkv.data_ptr(), B, NT, H, 64, 0.125, st) == 0


def ev(fn, reps=3):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


outs = []
for L in libs:
    fwd(L)
    bwd(L)
    torch.cuda.synchronize()
    outs.append((o.clone(), dqkv.clone()))
for i in range(1, len(libs)):
    print(f"{names[i]} vs {names[0]}: o equal {torch.equal(outs[0][0], outs[i][0])}, dqkv equal "
          f"{torch.equal(outs[0][1], outs[i][1])}, max |d dqkv| {float((outs[0][1].float() - outs[i][1].float()).abs().max())}",
          flush=True)
t = {(i, k): [] for i in range(len(libs)) for k in ("fwd", "bwd")}
for r in range(rounds):
    for i, L in enumerate(libs):
        fwd(L)
        t[(i, "fwd")].append(ev(lambda: fwd(L)))
        t[(i, "bwd")].append(ev(lambda: bwd(L)))
for i in range(len(libs)):
    f = sorted(t[(i, "fwd")])
    b = sorted(t[(i, "bwd")])
    print(f"{names[i]:28s} fwd med {f[rounds // 2]:.3f} min {f[0]:.3f} | bwd med {b[rounds // 2]:.3f} min {b[0]:.3f} ms",
          flush=True)
