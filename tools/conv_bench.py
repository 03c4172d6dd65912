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
    ap.add_argument("--kh", type=int, default=3)
    ap.add_argument("--kw", type=int, default=3)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--pad", type=int, default=-1, help="default: kernel // 2")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--act", type=int, default=0)
    ap.add_argument("--split", type=int, default=1, help="split_k (igemm partials, or conv_small's in-kernel split)")
    a = ap.parse_args()
    from tests.helpers import TORCH_DT, conv_op
    g = torch.Generator().manual_seed(0)
    dt = TORCH_DT[a.dtype]
    ph, pw = (a.kh // 2, a.kw // 2) if a.pad < 0 else (a.pad, a.pad)
    Ho = (a.hw + 2 * ph - a.kh) // a.stride + 1
    Wo = (a.hw + 2 * pw - a.kw) // a.stride + 1
    x = torch.randn(a.batch, a.hw, a.hw, a.cin, generator=g).to(dt).cuda()
    w = torch.randn(a.cout, a.cin, a.kh, a.kw, generator=g) / np.sqrt(a.kh * a.kw * a.cin)
    bias = torch.randn(a.cout, generator=g) * 0.1
    res = torch.randn(a.batch, Ho, Wo, a.cout, generator=g).to(dt).cuda() if a.res else None
    y = torch.empty(a.batch, Ho, Wo, a.cout, dtype=dt, device="cuda")
    tile = None if a.tile < 0 else a.tile
    kw = dict(stride=(a.stride, a.stride), pad=(ph, pw), bias=bias, res=res, y=y, tile=tile, dtype=a.dtype, act=a.act, split_k=a.split)
    conv_op(x, w, timed_iters=3, **kw)
    _, ms = conv_op(x, w, timed_iters=a.iters, **kw)
    us = float(np.median(ms)) * 1e3
    flop = 2.0 * a.batch * Ho * Wo * a.cout * a.kh * a.kw * a.cin
    print(json.dumps({"hw": a.hw, "cin": a.cin, "cout": a.cout, "k": [a.kh, a.kw], "stride": a.stride, "tile": a.tile, "split": a.split, "batch": a.batch,
                      "us": round(us, 1), "tflops": round(flop / us / 1e6, 1)}))


if __name__ == "__main__":
    main()
