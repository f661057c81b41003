"""A/B attention kernel variants selected by dclip_set_option, in ONE process (interleaved
rounds, same device, same random data) at the benchmark shape (B 8, H 12, N 8193, bf16).

  python tools/attn_opt_ab.py [-r ROUNDS] "8=0" "8=1" ...   (each arg: id=value[,id=value])
Prints per-variant fwd / bwd ms (median over rounds) and whether outputs match variant 0.
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseclip_vit_multimodal_amd import _native, ops  # noqa: E402

B, NT, C, H = 8, 8193, 768, 12
args = sys.argv[1:]
rounds = 7
if args and args[0] == "-r":
    rounds = int(args[1])
    args = args[2:]
variants = [dict(tuple(map(int, kv.split("="))) for kv in a.split(",") if kv) for a in (args or ["8=0"])]
L = _native.load()
torch.manual_seed(0)
qkv = torch.randn(B * NT, 3 * C, device="cuda").to(torch.bfloat16)
qkv[:, :C] = (qkv[:, :C].float() * 0.125 * 1.4426950408889634).to(torch.bfloat16)
dout = torch.randn(B * NT, C, device="cuda").to(torch.bfloat16)


def setv(v):
    for k in range(9):
        L.dclip_set_option(k, 0)
    for k, val in v.items():
        assert L.dclip_set_option(k, val) == 0


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
for v in variants:
    setv(v)
    o, lse = ops.attn_fwd(qkv, B, NT, H, 0.125)
    d = ops.attn_bwd(qkv, o, dout, lse, B, NT, H, 0.125)
    torch.cuda.synchronize()
    outs.append((o, lse, d))
for i in range(1, len(variants)):
    o0, l0, d0 = outs[0]
    o1, l1, d1 = outs[i]
    err = float((d1.float() - d0.float()).norm() / d0.float().norm())
    print(f"variant {variants[i]} vs {variants[0]}: o equal {torch.equal(o0, o1)}, dqkv equal {torch.equal(d0, d1)} "
          f"(rel diff {err:.2e})", flush=True)
o, lse, _ = outs[0]
times = {i: ([], []) for i in range(len(variants))}
for r in range(rounds):
    for i, v in enumerate(variants):
        setv(v)
        times[i][0].append(ev(lambda: ops.attn_fwd(qkv, B, NT, H, 0.125)))
        times[i][1].append(ev(lambda: ops.attn_bwd(qkv, o, dout, lse, B, NT, H, 0.125)))
fl = 4.0 * B * H * NT * NT * 64
for i, v in enumerate(variants):
    f, b = statistics.median(times[i][0]), statistics.median(times[i][1])
    print(f"variant {v}: fwd {f:.3f} ms ({fl / f / 1e9:.0f} TF/s), bwd {b:.3f} ms ({2.5 * fl / b / 1e9:.0f} TF/s useful)",
          flush=True)
