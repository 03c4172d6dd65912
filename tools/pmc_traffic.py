#!/usr/bin/env python3
"""HBM traffic per launch of the bench's kernel classes from rocprofv3 PMC passes.

Run on the GPU box after two SEPARATE counter passes of the bench command (never combined with a
tracing domain; FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950):
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf -o run -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw -o run -- python bench.py ...
    python tools/pmc_traffic.py --fetch gpurun_out/pf --write gpurun_out/pw --out profiles/r01_pmc_traffic.json

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts exactly half the bytes of 16-B/lane streaming reads (global_load and
buffer_load...lds alike), so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.  Both are the
L2's memory-side requests, i.e. Infinity-Cache hits are included (an upper bound on HBM bytes).
"""
import argparse
import csv
import glob
import json
import re
from collections import defaultdict

# bench/engine kernel class (fr_prof_get names) -> rocprof kernel-name prefix
BAND_VARIANT = {0: (2, 4, 7, 4), 1: (2, 4, 7, 2), 2: (4, 2, 4, 2)}
BAND_TH = {14: 14, 28: 7, 56: 4, 112: 2}


def class_pattern(cls: str, f16: bool) -> str:
    if cls == "stage layer3":  # the 13-fragment default (FR_OPT_STAGE_VARIANT 1: "::stage_kernel<")
        return f"stage13_kernel<{str(f16).lower()}>"
    if cls == "stage8 layer3":
        return "stage8_kernel("
    m = re.match(r"conv3x3_band W(\d+) v(\d+)", cls)
    if m:
        W, v = int(m.group(1)), int(m.group(2))
        if v == 3:  # software-pipelined 4-wave variant
            return f"conv3x3_bandp_kernel<{str(f16).lower()}, {W}, {BAND_TH[W]}, 2, 2, 7, 8,"
        wm, wn, fm, fn = BAND_VARIANT[v]
        return f"conv3x3_band_kernel<{str(f16).lower()}, {W}, {BAND_TH[W]}, {wm}, {wn}, {fm}, {fn},"
    raise KeyError(cls)


def per_kernel(root: str, counter: str):
    tot, n = defaultdict(float), defaultdict(int)
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"]
            tot[k] += float(r["Counter_Value"])
            n[k] += 1
    return {k: (tot[k], n[k]) for k in tot}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--arch", default="iresnet100")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--classes", nargs="*", default=["stage layer3", "conv3x3_band W14 v3"])
    ap.add_argument("--flops-per-launch", type=float, default=2.0 * 50176 * 256 * 2304,
                    help="algorithmic FLOPs per launch of the first class (intensity report)")
    a = ap.parse_args()
    fetch, write = per_kernel(a.fetch, "FETCH_SIZE"), per_kernel(a.write, "WRITE_SIZE")
    out = {"arch": a.arch, "dtype": a.dtype, "batch": a.batch, "kernels": {},
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes); bytes = 2*FETCH_SIZE*1024 + "
                     "WRITE_SIZE*1024 per dispatch (gfx950 FETCH_SIZE half-count correction)"}
    for cls in a.classes:
        pat = class_pattern(cls, a.dtype == "f16")
        fk = [k for k in fetch if k.startswith("void fr::") and pat in k] or [k for k in fetch if pat in k]
        wk = [k for k in write if pat in k]
        if not fk or not wk:
            print(f"{cls}: no dispatches matching {pat!r}")
            continue
        fb = sum(fetch[k][0] for k in fk) / sum(fetch[k][1] for k in fk) * 1024 * 2
        wb = sum(write[k][0] for k in wk) / sum(write[k][1] for k in wk) * 1024
        out["kernels"][cls] = {"rocprof_kernel": fk[0].split("(fr::")[0], "fetch_bytes_per_launch": round(fb),
                               "write_bytes_per_launch": round(wb), "hbm_bytes_per_launch": round(fb + wb),
                               "dispatches": sum(fetch[k][1] for k in fk)}
        print(cls, out["kernels"][cls])
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
