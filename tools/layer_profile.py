#!/usr/bin/env python3
"""Per-layer roofline view of one forward: run under
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python tools/layer_profile.py --run
then `python tools/layer_profile.py --trace DIR/run_kernel_trace.csv --plan DIR/plan.txt` aligns the
dispatches of the last forward with the plan (fr_debug_plan) and prints TFLOP/s per conv launch."""
import argparse
import csv
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(arch, dtype, B, iters, plan_path):
    import torch
    from facerecognition_amd import _native as N
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic(arch, max_batch=B, dtype=dtype)
    x = torch.from_numpy(synthetic_crops(B, m.input_size)).cuda()
    for _ in range(iters):
        m.embed(x)
    torch.cuda.synchronize()
    buf = ctypes.create_string_buffer(1 << 20)
    N.check(N.lib().fr_debug_plan(m.handle, B, buf, len(buf)), "fr_debug_plan")
    open(plan_path, "w").write(buf.value.decode())


def analyse(trace, plan_path):
    plan = [l.split() for l in open(plan_path).read().splitlines() if l.strip()]
    rows = list(csv.DictReader(open(trace)))
    ours = [r for r in rows if "fr::" in r["Kernel_Name"]]
    starts = [i for i, r in enumerate(ours)
              if any(k in r["Kernel_Name"] for k in ("preprocess", "stem_u8", "stem160"))]
    seq = ours[starts[-1]:]
    i = 0
    fused_stem = "stem_u8" in seq[0]["Kernel_Name"]
    if "stem160" in seq[0]["Kernel_Name"]:  # the IRV1 fused stem prepares u8 crops itself: no preprocess dispatch
        plan = [p for p in plan if p[0] != "pre"]
    skip_next_conv = False
    tot_ns = tot_flop = 0
    agg = {}
    per = []
    print(f"{'layer':34s} {'M':>8s} {'N':>5s} {'K':>5s} tile split {'us':>8s} {'TF/s':>7s}")
    for p in plan:
        if p[0] == "pre" and fused_stem:  # one dispatch = preprocess + the stem conv
            skip_next_conv = True
            continue
        if p[0] in ("pre", "maxpool", "avgpool"):
            r = seq[i]; i += 1
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            tot_ns += d
            print(f"{p[0]:34s} {'':>8s} {'':>5s} {'':>5s}           {d / 1e3:8.1f}")
            continue
        M, Nn, K, Kpad, tile, split = map(int, p[1:7])
        if skip_next_conv:
            p = ["stem", M, Nn, K, Kpad, tile, split, "stem(u8 fused)"]
            skip_next_conv = False
        d = 0
        r = seq[i]; i += 1
        d += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if p[0] == "chain" and "bneck28" in r["Kernel_Name"]:  # one launch per block
            for _ in range(tile - 1):
                r = seq[i]; i += 1
                d += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        elif (split > 1 and tile != 16) or p[0] == "head":  # (tile 16 = conv_small: its split is in-kernel)
            r = seq[i]; i += 1  # split-K epilogue / head finalize
            d += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        flop = 2.0 * M * Nn * K * (tile if p[0] in ("stage", "chain") else 1)  # stage: conv count, chain: blocks
        tot_ns += d
        tot_flop += flop
        key = (M, Nn, K, p[7])
        per.append((p[8] if len(p) > 8 else "-", p[0], M, Nn, K, tile, split, d, flop))
        agg.setdefault(key, [0, 0, 0.0, tile, split])
        agg[key][0] += 1
        agg[key][1] += d
        agg[key][2] += flop
    for (M, Nn, K, kk), (cnt, d, flop, tile, split) in sorted(agg.items(), key=lambda t: -t[1][1]):
        print(f"{kk + ' x' + str(cnt):34s} {M:8d} {Nn:5d} {K:5d} {tile:4d} {split:5d} {d / 1e3:8.1f} {flop / d / 1e3:7.1f}")
    print(f"forward: {tot_ns / 1e3:.1f} us, {tot_flop / tot_ns / 1e3:.1f} TFLOP/s over conv+head FLOPs")
    print("\nper launch (slowest first):")
    for name, kind, M, Nn, K, tile, split, d, flop in sorted(per, key=lambda t: -t[7]):
        print(f"  {name:24s} {kind:5s} {M:8d} {Nn:5d} {K:5d} {tile:4d} {split:5d} {d / 1e3:8.1f} {flop / d / 1e3:7.1f}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--arch", default="iresnet100")
    ap.add_argument("--dtype", default=None)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--plan", default="plan.txt")
    ap.add_argument("--trace")
    a = ap.parse_args()
    if a.run:
        run(a.arch, a.dtype, a.batch, a.iters, a.plan)
    else:
        analyse(a.trace, a.plan)
