#!/usr/bin/env python3
"""Face-logit offsets of the calibrated synthetic MTCNN weights (face_detector.CALIBRATED_LOGIT_SHIFT).

synth_mtcnn_state's random heads call 92 % of a smooth synthetic 1080p frame's 362k P-net windows a face, and
R-net / O-net pass most of what reaches them: every stage then carries 10^5 boxes, where a trained MTCNN on a
frame with a few faces carries ~10^3 P-net windows, ~10^2 R-net and ~10 O-net boxes.  This script measures,
with the CPU oracle nets (oracle/mtcnn.py) on tools/mtcnn_bench.py's frame, the (face - background) logit
quantiles at each stage and prints the offsets that make P-net pass ~1 % of windows, R-net ~10 % and O-net
~30 % of their inputs (assumed pass rates of a trained detector; parity unpinned: no reference fixture).

    python tools/calibrate_mtcnn.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

PASS = (0.01, 0.10, 0.30)


def main():
    from mtcnn_bench import frame
    from facerecognition_amd import face_detector as FD
    from oracle import mtcnn as OM
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    img = frame()
    th = [np.log(t / (1 - t)) for t in FD.THRESHOLDS]  # softmax pair: p(face) >= t <=> d >= log(t / (1 - t))
    st = FD.synth_mtcnn_state(7)
    shifts = []
    for stage, (key, p) in enumerate(zip(("pnet.conv4_1.bias", "rnet.dense5_1.bias", "onet.dense6_1.bias"), PASS)):
        ds = stage_logits(img, st, stage, FD, OM)
        delta = float(np.quantile(ds, 1 - p) - th[stage])
        shifts.append((key, round(delta, 2)))
        st[key] = st[key] + np.array([delta / 2, -delta / 2], np.float32)
        print(f"{key}: {len(ds)} inputs, offset {delta:.2f} -> pass {np.mean(ds - delta >= th[stage]):.3f}", flush=True)
    print("CALIBRATED_LOGIT_SHIFT =", {k: v for k, v in shifts})


def stage_logits(img, st, stage, FD, OM):
    """(face - background) logits of every input of `stage` (0 P, 1 R, 2 O) under weights st, the earlier
    stages run through the oracle's detect_face bookkeeping."""
    pnet, rnet, onet = OM.build_nets(st)
    H, W = img.shape[:2]
    x = torch.as_tensor(img).permute(2, 0, 1)[None].float()
    caught = {}

    def hook(name):
        def f(mod, inp, out):
            caught.setdefault(name, []).append((out[:, 1] - out[:, 0]).detach().flatten().numpy())
        return f
    layer = (pnet.conv4_1, rnet.dense5_1, onet.dense6_1)[stage]
    h = layer.register_forward_hook(hook("d"))
    with torch.no_grad():
        if stage == 0:
            for s in FD.pyramid_scales(H, W):
                im = (OM.imresample(x, (int(H * s + 1), int(W * s + 1))) - 127.5) * 0.0078125
                pnet(im)
        else:
            OM.detect_face(img[None], pnet, rnet, onet)
    h.remove()
    return np.concatenate(caught.get("d", [np.zeros(0, np.float32)]))


if __name__ == "__main__":
    main()
