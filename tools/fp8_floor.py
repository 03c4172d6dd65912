#!/usr/bin/env python3
"""Accuracy floor of fp8 weights for BASELINE config 5, measured on the fp32 oracle (CPU, no GPU):
IResNet100 with every conv weight of >= 64 input channels fake-quantized to OCP e4m3 with a per-output-
channel scale (the quantizer of weights.quantize_fp8), activations kept in fp32.  Any fp8-weight
implementation, whatever its activation precision, carries at least this error.

    python tools/fp8_floor.py [--n 4]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def e4m3_per_channel(w):
    w = torch.as_tensor(np.asarray(w, dtype=np.float32))
    amax = w.abs().reshape(w.shape[0], -1).amax(dim=1)
    s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax)).view((-1,) + (1,) * (w.dim() - 1))
    return ((w / s).clamp(-448, 448).to(torch.float8_e4m3fn).float() * s).numpy()


def main():
    from facerecognition_amd.synthetic import synthetic_crops
    from facerecognition_amd.weights import synth_state_dict
    from oracle import models as M
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4)
    a = ap.parse_args()
    sd = synth_state_dict("iresnet100")
    u8 = synthetic_crops(a.n, 112, seed=4)
    ref = M.embed(M.build_model("iresnet100", sd), "iresnet100", u8)
    sdq = {k: (e4m3_per_channel(v) if k.endswith("weight") and np.asarray(v).ndim == 4 and np.asarray(v).shape[1] % 64 == 0
               else v) for k, v in sd.items()}
    q = M.embed(M.build_model("iresnet100", sdq), "iresnet100", u8)
    cos = (q * ref).sum(1) / np.linalg.norm(q, axis=1) / np.linalg.norm(ref, axis=1)
    print("IResNet100, e4m3 per-channel weights, fp32 activations: 1-cos =", np.round(1 - cos, 5))


if __name__ == "__main__":
    main()
