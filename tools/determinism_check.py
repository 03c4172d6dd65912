#!/usr/bin/env python3
"""Replay determinism at full batch: embed the same bs=256 batch N times and report which calls differ
(call 0 runs the tile-tuning pass).  Use with env toggles (FR_AB=no_img28, FR_AB=no_stage, ...) to
isolate a kernel."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    m = FRModel.synthetic("iresnet100", dtype="bf16")
    u8 = torch.from_numpy(synthetic_crops(256, 112, seed=21))
    outs = [m.embed(u8).cpu() for _ in range(n)]
    for i in range(1, n):
        d = (outs[i] - outs[1]).abs().max().item()
        rows = int(((outs[i] - outs[1]).abs().amax(1) > 0).sum())
        print(f"call {i} vs 1: max diff {d:.3e}, rows differing {rows}")
    d0 = (outs[0] - outs[1]).abs().max().item()
    print(f"call 0 (tuning pass) vs 1: max diff {d0:.3e}")


if __name__ == "__main__":
    main()
