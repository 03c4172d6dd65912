#!/usr/bin/env python3
"""FaceNet IRV1 LDS-resident blocks (conv_block.hip) vs their member convs: the measured per-block choice of the
tuning forward (fr_debug_plan's block lines carry "<block ms> <per-conv ms>"), then whole-forward timings with
the blocks forced on (FR_OPT_STAGE 2) and off (0), HIP events over graph replays.

    python tools/block_ab.py [--batch 256] [--iters 20]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from facerecognition_amd import _native as N
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--arch", default="irv1_facenet")
    a = ap.parse_args()
    B = a.batch
    m = FRModel.synthetic(a.arch, max_batch=B)
    x = torch.from_numpy(synthetic_crops(B, m.input_size)).cuda()
    m.embed(x)
    torch.cuda.synchronize()
    buf = ctypes.create_string_buffer(1 << 20)
    N.check(N.lib().fr_debug_plan(m.handle, B, buf, len(buf)), "fr_debug_plan")
    for l in buf.value.decode().splitlines():
        if l.startswith(("block", "stage")):
            print("plan:", l, flush=True)
    for mode in (1, 2, 0, 2, 0):
        m.set_option(N.FR_OPT_STAGE, mode)
        for _ in range(3):
            m.embed(x)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            m.embed(x)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        print(f"FR_OPT_STAGE={mode}: {ms:.4f} ms/forward, {B / ms * 1e3:.0f} faces/s", flush=True)


if __name__ == "__main__":
    main()
