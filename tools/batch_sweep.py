"""Forward latency vs batch size, per-conv launches vs the layer3 stage kernel (FR_OPT_STAGE 0 / 2) and
the auto rule (1).  One JSON line per (B, mode): median ms of `--iters` graph replays, inputs in HBM.
    python tools/batch_sweep.py [--arch iresnet100] [--batches 1,8,64,128,256]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="iresnet100")
    ap.add_argument("--dtype", default=None)
    ap.add_argument("--batches", default="1,2,4,8,16,32,64,96,128,160,192,208,224,240,256")
    ap.add_argument("--modes", default="0,2,1")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from facerecognition_amd import _native as N
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic(a.arch, max_batch=256, dtype=a.dtype)
    x_all = torch.from_numpy(synthetic_crops(256, m.input_size, seed=3)).cuda()
    out = torch.empty((256, 512), dtype=torch.float32, device="cuda")
    for B in [int(b) for b in a.batches.split(",")]:
        x = x_all[:B].contiguous()
        o = out[:B]
        for mode in [int(v) for v in a.modes.split(",")]:
            m.set_option(N.FR_OPT_STAGE, mode)
            for _ in range(3):  # tune + capture + replay
                m.embed(x, out=o)
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.iters):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                m.embed(x, out=o)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = float(np.median(ts))
            print(json.dumps({"arch": a.arch, "dtype": m.dtype, "B": B, "stage_mode": mode, "ms": round(ms, 4),
                              "faces_per_s": round(B / ms * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
