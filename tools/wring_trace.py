#!/usr/bin/env python3
"""Phase timing of conv_wring from its FR_WRING_TRACE build (timing experiment only): the last wring launch of
an IResNet100 forward (layer4.2.conv2: 12544 x 512 x 4608, 36 stages of 128 channels):

    tools/build_variant.sh wtrace "-DFR_WRING_TRACE"
    FR_LIBFRHIP=facerecognition_amd/lib/variants/libfrhip_wtrace.so python tools/wring_trace.py

Per wave of two blocks: prologue, per-stage period (barrier to barrier), time in the stage-boundary wait
(vmcnt + barrier), the main loop end to the kernel end (epilogue), in shader clocks."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ST, NT = 40, 4 + 2 * 40


def main():
    from facerecognition_amd import _native as N
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    L = N.lib()
    m = FRModel.synthetic("iresnet100")
    x = torch.from_numpy(synthetic_crops(256, 112, seed=3)).cuda()
    for _ in range(3):
        m.embed(x)
    torch.cuda.synchronize()
    buf = (ctypes.c_uint * (2 * 8 * NT))()
    L.fr_wring_trace_read.restype = ctypes.c_int
    assert L.fr_wring_trace_read(buf, len(buf)) == len(buf)
    t = np.frombuffer(buf, dtype=np.uint32).reshape(2, 8, NT).astype(np.int64)
    t = t - t[:, :1, :1]
    t = np.where(t < -(1 << 31), t + (1 << 32), t)
    nst = 36
    for b in range(2):
        print(f"block {'0' if b == 0 else '100'}:")
        for w in (0, 3, 4, 7):
            r = t[b, w]
            bar = r[3:3 + 2 * nst:2]
            pre = r[2:2 + 2 * nst:2]
            per = np.diff(bar)
            wait = bar - pre
            print(f"  wave {w}: prologue {r[1] - r[0]:6d}  stage period mean {per.mean():7.0f} (min {per.min()}, max {per.max()})"
                  f"  boundary wait mean {wait.mean():6.0f}  loop {r[NT - 2] - r[1]:7d}  epilogue {r[NT - 1] - r[NT - 2]:6d}"
                  f"  total {r[NT - 1] - r[0]:7d}")
    print("MFMA floor per stage per SIMD: 2 waves x 4 substeps x 14 MFMAs x 16 cycles = 1792 cycles")
    m.close()


if __name__ == "__main__":
    main()
