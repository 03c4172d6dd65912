#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc CSVs (tools/pmc_run.sh output) per kernel name: sums and per-dispatch means."""
import csv
import glob
import sys
from collections import defaultdict


def main(root, filt=""):
    agg = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if filt not in k:
                continue
            key = k.split("(")[0][-70:]
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[key][r["Counter_Name"]] += 1
    for k, d in agg.items():
        print(k)
        n = max(cnt[k].values())
        for c in sorted(d):
            print(f"   {c:28s} total {d[c]:.4g}   per-dispatch {d[c] / cnt[k][c]:.4g}   (n={cnt[k][c]})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
