#!/usr/bin/env python3
"""Phase timing of the layer3 stage kernel from its FR_STAGE_TRACE build (timing experiment only):

    tools/build_variant.sh trace "-DFR_STAGE_TRACE"
    FR_LIBFRHIP=facerecognition_amd/lib/variants/libfrhip_trace.so python tools/stage_trace.py [--batch 256]

Per conv and wave of two workgroups: K loop, wait at the epilogue's entry barrier, epilogue (to the exit
barrier), and the gap to the next conv's K loop (seed / table loads / output copy), in shader clocks."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    from facerecognition_amd import _native as N
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    L = N.lib()
    m = FRModel.synthetic("iresnet100", dtype=args.dtype)
    x = torch.from_numpy(synthetic_crops(args.batch, 112, seed=3)).cuda()
    for _ in range(3):
        m.embed(x)
    torch.cuda.synchronize()
    n = 2 * 8 * 16 * 4
    buf = (ctypes.c_uint * n)()
    L.fr_stage_trace_read.restype = ctypes.c_int
    got = L.fr_stage_trace_read(buf, n)
    assert got == n, got
    t = np.frombuffer(buf, dtype=np.uint32).reshape(2, 8, 16, 4).astype(np.int64)
    t = t - t[:, :1, :1, :1]
    t = np.where(t < -(1 << 31), t + (1 << 32), t)  # 32-bit clock wrap
    for wg in range(2):
        print(f"workgroup {'0' if wg == 0 else '200'}: per conv (cycles) kloop / entry-wait / epilogue / gap-to-next")
        for w in (0, 3, 4, 7):
            rows = []
            for cv in range(1, 15):
                k = t[wg, w, cv, 1] - t[wg, w, cv, 0]
                e_w = t[wg, w, cv, 2] - t[wg, w, cv, 1]
                ep = t[wg, w, cv, 3] - t[wg, w, cv, 2]
                gap = t[wg, w, cv + 1, 0] - t[wg, w, cv, 3]
                rows.append((k, e_w, ep, gap))
            r = np.array(rows)
            tot = r.sum(axis=1)
            print(f"  wave {w}: kloop {r[:, 0].mean():8.0f}  wait {r[:, 1].mean():6.0f}  epi {r[:, 2].mean():6.0f}  "
                  f"gap {r[:, 3].mean():6.0f}  per conv {tot.mean():8.0f}  (kloop share {r[:, 0].sum() / tot.sum():.3f})")
    # clock: conv period in cycles vs the bench's per-conv time
    per = np.diff(t[0, 0, 1:15, 0]).mean()
    print(f"conv period (wave 0, wg 0): {per:.0f} cycles")
    m.close()


if __name__ == "__main__":
    main()
