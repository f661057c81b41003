"""Probe: which BatchNorm2d calls crash on the box (each case in its own child process).
  python tools/bn_probe.py            # parent: runs every case, prints exit codes
  python tools/bn_probe.py CASE       # child: one case"""
import subprocess
import sys

CASES = [(b, h, w, dt, cl, miopen) for (b, h, w) in [(1, 64, 128), (1, 73, 146), (8, 73, 146), (1, 73, 148)]
         for dt in ("bf16", "f32") for cl in (1, 0) for miopen in (1, 0)]


def child(i):
    import torch
    b, h, w, dt, cl, miopen = CASES[i]
    x = torch.randn(b, 128, h, w, device="cuda", dtype=torch.bfloat16 if dt == "bf16" else torch.float32)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    bn = torch.nn.BatchNorm2d(128).cuda().train()
    with torch.backends.cudnn.flags(enabled=bool(miopen)):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(dt == "bf16")):
            y = bn(x)
        y.float().sum().backward()
    torch.cuda.synchronize()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(int(sys.argv[1]))
        sys.exit(0)
    for i, c in enumerate(CASES):
        r = subprocess.run([sys.executable, __file__, str(i)], capture_output=True, text=True, timeout=120)
        print(c, "rc", r.returncode, r.stderr.strip().splitlines()[-1][:150] if r.returncode else "", flush=True)
