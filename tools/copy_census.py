"""Census of torch's element-wise kernels in a rocprofv3 kernel trace: grouped by (kind, grid size,
stream), with calls, total and mean durations, so the copies / adds of a step can be traced to
their tensors (grid size = elements / 4 per thread for the unrolled kernels).

  python tools/copy_census.py <kernel_trace.csv> [steps]
"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
agg = defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"]
    if "at::native" not in n:
        continue
    if "direct_copy" in n:
        kind = "copy"
    elif "CUDAFunctor_add" in n or "AddFunctor" in n:
        kind = "add"
    elif "FillFunctor" in n:
        kind = "fill"
    elif "MulFunctor" in n:
        kind = "mul"
    else:
        kind = n.split("<")[0][-40:]
    kind += ("/unroll" if "manual_unroll" in n else "/vec" if "vectorized" in n else "")
    for t in ("float)", "double)", "unsigned char)", "c10::BFloat16)", "c10::Half)", "long)"):
        if "lambda(" + t in n:
            kind += "/" + t[:-1]
            break
    grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
    key = (kind, grid, r.get("Stream_Id", r.get("Queue_Id", "?")))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    agg[key][0] += 1
    agg[key][1] += d
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
print(f"{'us/step':>9} {'calls/st':>8} {'mean us':>8}  kind / grid / stream")
for (kind, grid, stream), (c, t) in rows[:40]:
    print(f"{t / steps:9.1f} {c / steps:8.1f} {t / c:8.1f}  {kind} / grid {grid} / stream {stream}")
