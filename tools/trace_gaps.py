#!/usr/bin/env python3
"""Timeline of the bench's steady-state steps from a rocprofv3 --kernel-trace CSV: per kernel of one step
its duration and the idle gap before it, and per step the sum of kernel time vs the step's span.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -o run -- python bench.py --steps 5 \
        --warmup 2 --no-cpu-baseline --no-prof --no-pmc
    python tools/trace_gaps.py gpurun_out/kt [--first stem_u8_kernel]
"""
import argparse
import csv
import glob
import re


def short(name):
    name = name.replace("void ", "").replace("fr::(anonymous namespace)::", "")
    name = re.sub(r"\(fr::.*|\(float const.*|\(unsigned.*", "", name)
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--first", default="stem_u8_kernel", help="kernel that starts a step")
    ap.add_argument("--steps", type=int, default=3, help="last N complete steps to report")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(f"{a.root}/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.first in r["Kernel_Name"]]
    if len(starts) < 2:
        raise SystemExit("fewer than two steps found")
    steps = [(starts[i], starts[i + 1]) for i in range(len(starts) - 1)][-a.steps:]
    for s, e in steps:
        seg = rows[s:e]
        t0 = int(seg[0]["Start_Timestamp"])
        t1 = int(seg[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
        print(f"step: {len(seg)} kernels, span {(t1 - t0) / 1e3:.1f} us, kernel time {busy / 1e3:.1f} us, "
              f"idle {(t1 - t0 - busy) / 1e3:.1f} us; next step starts +{(int(rows[e]['Start_Timestamp']) - t1) / 1e3:.1f} us")
    s, e = steps[-1]
    prev = None
    print(f"{'kernel':70s} {'us':>8s} {'gap us':>8s}")
    for r in rows[s:e]:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (st - prev) / 1e3 if prev is not None else 0.0
        print(f"{short(r['Kernel_Name']):70s} {(en - st) / 1e3:8.1f} {gap:8.1f}")
        prev = en


if __name__ == "__main__":
    main()
