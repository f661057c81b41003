"""Where DDP's gradient all-reduce kernels fall inside a train step, from a rocprofv3 kernel trace.

  python tools/ddp_trace.py <run_kernel_trace.csv> [--out profiles/<name>.txt]

The last step of the trace is the span from the last patch-embedding im2col launch (the first
kernel of a forward) to the end.  For that step it lists every RCCL kernel (all-reduce of a DDP
bucket) with its start / end relative to the step start, the backward's span (first to last
attention-backward launch), how much of each all-reduce overlaps other kernels running at the
same time, and the step's kernel-busy time.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "im2col" in r["Kernel_Name"]]
    if not starts:
        raise SystemExit("no im2col launch in the trace")
    step = rows[starts[-1]:]
    t0 = int(step[0]["Start_Timestamp"])
    iv = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Kernel_Name"]) for r in step]
    t_end = max(e for _, e, _ in iv)
    comm = [x for x in iv if "nccl" in x[2].lower() or "rccl" in x[2].lower()]
    bwd = [x for x in iv if "attn_bwd" in x[2]]
    other = [x for x in iv if x not in comm]

    def overlap(s, e):
        # time of [s, e) during which at least one non-RCCL kernel runs
        segs = sorted((max(s, a), min(e, b)) for a, b, _ in other if a < e and b > s)
        tot, cur_s, cur_e = 0, None, None
        for x, y in segs:
            if cur_e is None or x > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = x, y
            else:
                cur_e = max(cur_e, y)
        if cur_e is not None:
            tot += cur_e - cur_s
        return tot

    lines = [f"step span {t_end / 1e6:.3f} ms, {len(iv)} kernels, {len(comm)} RCCL kernels"]
    if bwd:
        lines.append(f"attention backward launches {len(bwd)}: first at {bwd[0][0] / 1e6:.3f} ms, "
                     f"last ends {bwd[-1][1] / 1e6:.3f} ms")
    tot_c = tot_o = 0
    for s, e, n in comm:
        o = overlap(s, e)
        tot_c += e - s
        tot_o += o
        lines.append(f"  RCCL {s / 1e6:9.3f} -> {e / 1e6:9.3f} ms  ({(e - s) / 1e3:8.1f} us, overlapped "
                     f"{o / max(1, e - s) * 100:5.1f} %)  {n[:90]}")
    if comm:
        lines.append(f"RCCL kernel time {tot_c / 1e6:.3f} ms, of it overlapped with compute {tot_o / 1e6:.3f} ms "
                     f"({tot_o / max(1, tot_c) * 100:.1f} %); after the last attention backward: "
                     f"{sum(e - max(s, bwd[-1][1]) for s, e, _ in comm if e > bwd[-1][1]) / 1e6 if bwd else 0:.3f} ms")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
