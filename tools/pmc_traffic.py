"""HBM traffic per launch of one kernel from rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE
in separate passes; both in KiB), with the gfx950 correction of MI355X_MICROARCH.md §HBM:
FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.

  python tools/pmc_traffic.py <pass dirs...> --kernel attn_fwd_kernel --algorithmic BYTES --out profiles/x.json
"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--algorithmic", type=float, required=True, help="algorithmic HBM bytes per launch")
    ap.add_argument("--out")
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    for d in a.dirs:
        try:
            rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
        except (FileNotFoundError, NotADirectoryError):
            continue
        for r in rows:
            if a.kernel in r["Kernel_Name"] and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
                per[r["Counter_Name"]][(d, r["Dispatch_Id"])] += float(r["Counter_Value"])
    mean = {c: sum(v.values()) / len(v) for c, v in per.items()}
    fetch = 2.0 * mean["FETCH_SIZE"] * 1024
    write = mean["WRITE_SIZE"] * 1024
    res = {"kernel": a.kernel, "hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
           "algorithmic_bytes": a.algorithmic, "ratio_to_algorithmic": (fetch + write) / a.algorithmic,
           "dispatches": {c: len(v) for c, v in per.items()},
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (KiB); FETCH_SIZE x2 (gfx950 "
                     "half-count of 16-B/lane reads, MI355X_MICROARCH.md)"}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
