"""Per-kernel summary (calls, total / mean / min ms) from a rocprofv3 sqlite database (rocpd_*):
  python tools/rocpd_stats.py gpurun_out/r6l/prof/run_results.db [--filter attn] [--csv out.csv]"""
import argparse
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--filter", default="")
    ap.add_argument("--csv", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("""select s.display_name, d.end - d.start from rocpd_kernel_dispatch d
                        join rocpd_info_kernel_symbol s on d.kernel_id = s.id""").fetchall()
    agg = {}
    for name, ns in rows:
        if a.filter and a.filter not in name:
            continue
        agg.setdefault(name, []).append(ns / 1e6)
    out = sorted(((sum(v), len(v), sum(v) / len(v), min(v), k) for k, v in agg.items()), reverse=True)
    lines = ["Name,Calls,TotalMs,AverageMs,MinMs"]
    for tot, n, avg, mn, k in out:
        lines.append(f'"{k}",{n},{tot:.4f},{avg:.4f},{mn:.4f}')
    print("\n".join(lines))
    if a.csv:
        open(a.csv, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    sys.exit(main())
