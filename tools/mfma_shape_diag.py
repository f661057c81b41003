"""A/B timing of the attention kernels: fwd / bwd launches at the bench shape (B=8, N=8193, H=12)
through the C ABI of the library given on the command line, per-launch HIP-event medians and a
bitwise fingerprint of dQKV (two builds that should agree bit for bit print the same number).
Run the libraries in separate processes, alternately (tools/gpu_r04j.sh).

  python tools/mfma_shape_diag.py path/to/lib.so [reps] [dtype code: 2 bf16 (default), 1 fp16]
"""
import ctypes
import sys

import torch

lib = ctypes.CDLL(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
DT = int(sys.argv[3]) if len(sys.argv) > 3 else 2  # DCLIP_BF16 (2) or DCLIP_F16 (1)
tdt = torch.float16 if DT == 1 else torch.bfloat16
B, N, H, D = 8, 8193, 12, 64
C = H * D
torch.manual_seed(0)
qkv = (torch.randn(B * N, 3 * C, device="cuda") * 0.5).to(tdt)
qkv[:, :C] *= 0.125 * 1.4426950408889634
dout = torch.randn(B * N, C, device="cuda").to(tdt)
o = torch.empty(B * N, C, device="cuda", dtype=tdt)
lse = torch.empty(B * H * N, device="cuda", dtype=torch.float32)
lib.dclip_attn_bwd_workspace.restype = ctypes.c_int64
ws = torch.empty(lib.dclip_attn_bwd_workspace(B, N, H), device="cuda", dtype=torch.float32)
dqkv = torch.empty_like(qkv)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = ctypes.c_void_p


def fwd():
    rc = lib.dclip_attn_fwd(DT, P(qkv.data_ptr()), P(o.data_ptr()), P(lse.data_ptr()), B, N, H, D,
                            ctypes.c_float(0.125), st)
    assert rc == 0, rc


def bwd():
    rc = lib.dclip_attn_bwd(DT, P(qkv.data_ptr()), P(o.data_ptr()), P(dout.data_ptr()), P(lse.data_ptr()),
                            P(ws.data_ptr()), P(dqkv.data_ptr()), B, N, H, D, ctypes.c_float(0.125), st)
    assert rc == 0, rc


def timed(fn):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


fwd()
tf = timed(fwd)
tb = timed(bwd)
bits = dqkv.view(torch.int16).long().flatten()
chk = int((bits * (torch.arange(bits.numel(), device="cuda") % 65521 + 1)).sum())  # bitwise fingerprint of dqkv
print(f"{sys.argv[1].split('/')[-1]} {tdt}: fwd {tf:.3f} ms  bwd {tb:.3f} ms  dqkv fingerprint {chk}  "
      f"finite o {bool(torch.isfinite(o.float()).all())} dqkv {bool(torch.isfinite(dqkv.float()).all())}", flush=True)
