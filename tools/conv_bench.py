#!/usr/bin/env python3
"""Time one conv through fr_op_conv2d at bs=256 with a forced kernel (HIP events on the launching
stream), e.g. the layer2 conv:  python tools/conv_bench.py --hw 28 --cin 128 --cout 128 --tile 10
(--tile: FR_TILE_* id; -1 = automatic).  Prints one JSON line with us/launch and TFLOP/s."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--hw", type=int, default=28)
    ap.add_argument("--cin", type=int, default=128)
    ap.add_argument("--cout", type=int, default=128)
    ap.add_argument("--tile", type=int, default=-1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--res", action="store_true", help="residual input (the conv2 epilogue)")
    a = ap.parse_args()
    from tests.helpers import conv_op
    g = torch.Generator().manual_seed(0)
    x = torch.randn(a.batch, a.hw, a.hw, a.cin, generator=g).to(torch.bfloat16).cuda()
    w = torch.randn(a.cout, a.cin, 3, 3, generator=g) / np.sqrt(9 * a.cin)
    bias = torch.randn(a.cout, generator=g) * 0.1
    res = torch.randn(a.batch, a.hw, a.hw, a.cout, generator=g).to(torch.bfloat16).cuda() if a.res else None
    y = torch.empty(a.batch, a.hw, a.hw, a.cout, dtype=torch.bfloat16, device="cuda")
    tile = None if a.tile < 0 else a.tile
    conv_op(x, w, pad=(1, 1), bias=bias, res=res, y=y, tile=tile, timed_iters=3)
    _, ms = conv_op(x, w, pad=(1, 1), bias=bias, res=res, y=y, tile=tile, timed_iters=a.iters)
    us = float(np.median(ms)) * 1e3
    flop = 2.0 * a.batch * a.hw * a.hw * a.cout * 9 * a.cin
    print(json.dumps({"hw": a.hw, "cin": a.cin, "cout": a.cout, "tile": a.tile, "us": round(us, 1),
                      "tflops": round(flop / us / 1e6, 1)}))


if __name__ == "__main__":
    main()
