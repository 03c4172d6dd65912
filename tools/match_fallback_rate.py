#!/usr/bin/env python3
"""Proof-fallback rate of the bf16 candidate match (match_x3.hip) over seeded random galleries: one search per
seed, the number of probes rescanned exactly (fr_debug_match_fallbacks delta) and the search time.

    python tools/match_fallback_rate.py [--rows 1000000 --probes 256 --seeds 8]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--probes", type=int, default=256)
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--k", type=int, default=5)
    a = ap.parse_args()
    from facerecognition_amd.gallery import DeviceGallery
    tot = 0
    for seed in range(a.seeds):
        torch.manual_seed(seed)
        g = torch.randn(a.rows, 512, device="cuda")
        g = g / g.norm(dim=1, keepdim=True)
        p = torch.randn(a.probes, 512, device="cuda")
        p = p / p.norm(dim=1, keepdim=True)
        gal = DeviceGallery(handle=None)
        gal.set_device_rows(g)
        fb0 = gal.fallbacks()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gal.search_device(p, a.k)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        fb = gal.fallbacks() - fb0
        tot += fb
        print(json.dumps({"seed": seed, "rows": a.rows, "probes": a.probes, "fallbacks": fb, "ms": round(ms, 3)}), flush=True)
        gal.close()
        del g, p
    print(json.dumps({"total_fallbacks": tot, "probe_searches": a.seeds * a.probes}), flush=True)


if __name__ == "__main__":
    main()
