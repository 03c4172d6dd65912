#!/usr/bin/env python3
"""Generate BN running statistics for the synthetic weights (run once, in this container).

SURVEY.md §0.5: with default BN statistics, random-weight embeddings collapse (pairwise cosine
0.99+), which makes every top-1 test meaningless.  One train-mode pass (momentum=None, dropout
kept in eval) over 64 synthetic crops (facerecognition_amd.synthetic, seed 7) of the oracle restatement gives
well-conditioned eval-mode statistics.  Output: facerecognition_amd/synth/<arch>_bnstats.npz,
consumed by facerecognition_amd.weights.synth_state_dict (weights themselves are regenerated
bit-exactly from the splitmix64 seed everywhere, so only these statistics are stored).
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from facerecognition_amd import weights as W  # noqa: E402
from facerecognition_amd.synthetic import synthetic_crops  # noqa: E402
from oracle import models as M  # noqa: E402


def main(archs=W.ARCHS, seed=1234, n=64):
    torch.set_num_threads(os.cpu_count() or 1)
    os.makedirs(W.SYNTH_DIR, exist_ok=True)
    for arch in archs:
        t = time.time()
        sd = W.synth_state_dict(arch, seed=seed, calibrated=False)
        model = M.build_model(arch, sd)
        s = W.INPUT_SIZE[arch]
        u8 = synthetic_crops(n, s, seed=7)
        stats = M.calibrate_bn(model, M.preprocess_u8_nhwc(u8))
        stats["__seed__"] = np.array(seed)
        np.savez_compressed(W.bnstats_path(arch), **stats)
        # sanity: embeddings of different random crops should be far apart after calibration
        sd2 = W.synth_state_dict(arch, seed=seed, calibrated=True)
        model2 = M.build_model(arch, sd2)
        e = M.embed(model2, arch, u8[:16])
        c = e @ e.T
        off = c[~np.eye(len(c), dtype=bool)]
        print(f"{arch}: {len(stats) - 1} stats, pairwise cos mean {off.mean():+.4f} max {off.max():+.4f} "
              f"({time.time() - t:.1f}s)")


if __name__ == "__main__":
    main(tuple(sys.argv[1:]) or W.ARCHS)
