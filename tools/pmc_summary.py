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
            key = k.replace("(anonymous namespace)::", "").rsplit("(", 1)[0][-90:]
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[key][r["Counter_Name"]] += 1
    for k, d in agg.items():
        print(k)
        n = max(cnt[k].values())
        for c in sorted(d):
            print(f"   {c:28s} total {d[c]:.4g}   per-dispatch {d[c] / cnt[k][c]:.4g}   (n={cnt[k][c]})")
        if d.get("SQ_WAVE_CYCLES"):  # quad-cycle counters over the same waves (MI355X_MICROARCH.md)
            w = d["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if c in d:
                    print(f"   {c + ' / SQ_WAVE_CYCLES':44s} {d[c] / w:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
