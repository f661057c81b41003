"""Summarise a rocprofv3 kernel-trace CSV over the steady-state region of a bench run.

  python tools/prof_summary.py <run_kernel_trace.csv> [--skip-marker attn_fwd_kernel --skip N]
      [--steps K] [--out profiles/<name>.txt]

The region starts at the (N+1)-th dispatch whose name contains the marker (e.g. skip the
warmup steps' attention forwards: N = warmup * 12) and runs to the end of the trace.
Prints per-kernel calls, total, mean, share of GPU busy time and per-step totals.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "")
    m = re.search(r"_ZN12_GLOBAL__N_1\d+(\w+?)I", n)
    if m:
        n = m.group(1) + n[n.find("I", m.end() - 1):][:40]
    return n[:100]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-marker", default="attn_fwd_kernel")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seen = 0
    start = None
    for i, r in enumerate(rows):
        if a.skip_marker in r["Kernel_Name"]:
            if seen == a.skip:
                start = i
                break
            seen += 1
    rows = rows[start or 0:]
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += d
    busy = sum(v[1] for v in agg.values())
    wall = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6
    lines = [f"region: {len(rows)} dispatches, GPU-busy {busy:.2f} ms, wall {wall:.2f} ms, steps {a.steps}",
             f"{'ms/step':>9} {'calls/st':>8} {'mean us':>9} {'share':>6}  kernel"]
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{t / a.steps:9.3f} {n / a.steps:8.1f} {t / n * 1e3:9.1f} {100 * t / busy:5.1f}%  {k}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
