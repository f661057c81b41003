"""Aggregate rocprofv3 --pmc counter_collection CSVs: per kernel (short name) the mean
value per dispatch of every counter found in the given pass directories."""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.search(r"_ZN12_GLOBAL__N_1\d+(\w+?)I", n)
    if m:
        return m.group(1)
    n = re.sub(r"^void ", "", n)
    return re.sub(r"[<(].*", "", n)[:40]


def main(dirs):
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
        per = defaultdict(float)
        for r in rows:
            per[(r["Dispatch_Id"], short(r["Kernel_Name"]), r["Counter_Name"])] += float(r["Counter_Value"])
        for (did, k, c), v in per.items():
            vals[k][c].append(v)
    for k, cs in vals.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:32s} {sum(v) / len(v):16.4e}   (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1:])
