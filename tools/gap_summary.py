"""GPU idle time inside the steady-state steps of a rocprofv3 kernel trace: the union of all
dispatch intervals (every queue) against the wall from the first to the last dispatch of the
region, and the largest idle gaps with the dispatches either side of them.

  python tools/gap_summary.py <kernel_trace.csv> --skip N [--marker attn_fwd2] [--steps K] [--top 25]
"""
import argparse
import csv
from collections import Counter

from prof_summary import short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="attn_fwd2")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    seen, start = 0, 0
    for i, r in enumerate(rows):
        if a.marker in r["Kernel_Name"]:
            if seen == a.skip:
                start = i
                break
            seen += 1
    rows = rows[start:]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows]
    busy, gaps = 0, []
    cur_s, cur_e, cur_k = iv[0]
    for s, e, k in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_k, k))
            cur_s, cur_e, cur_k = s, e, k
        elif e > cur_e:
            cur_e, cur_k = e, k
    busy += cur_e - cur_s
    wall = iv[-1][1] - iv[0][0]
    idle = sum(g[0] for g in gaps)
    print(f"region {len(iv)} dispatches, wall {wall / 1e6:.2f} ms, GPU busy (union) {busy / 1e6:.2f} ms "
          f"= {100 * busy / wall:.1f} %, idle {idle / 1e6:.2f} ms ({idle / 1e6 / a.steps:.3f} ms per step)")
    by_pair = Counter()
    for g, k0, k1 in gaps:
        by_pair[(k0[:50], k1[:50])] += g
    print(f"idle per step by (before -> after), top {a.top}:")
    for (k0, k1), g in by_pair.most_common(a.top):
        print(f"  {g / 1e3 / a.steps:9.1f} us  {k0}  ->  {k1}")


if __name__ == "__main__":
    main()
