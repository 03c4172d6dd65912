#!/usr/bin/env python3
"""fp8 activation-scale granularity on the CPU fake-quant model of tools/fp8_plan.py: one power-of-two scale
per image and conv input (conv_stage8.hip) vs one per (pixel, 32-channel K-block) (the e8m0 B-operand block
scales of v_mfma_scale_f32_16x16x128_f8f6f4), for three conv sets.  profiles/r04_fp8_mx32_sensitivity.txt."""
import os, sys, torch, torch.nn.functional as F, numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tools"))
import fp8_plan as P
from facerecognition_amd.synthetic import synthetic_crops
from facerecognition_amd.weights import synth_state_dict
from oracle import models as M
torch.set_num_threads(8)
model = M.build_model("iresnet100", synth_state_dict("iresnet100")).eval()
xin = M.preprocess_u8_nhwc(synthetic_crops(8, 112, seed=4))
with torch.no_grad(): ref = P.forward_q(model, xin, set())
def q_mx(x):  # per (pixel, 32-channel group) power-of-two scale
    B, C, H, W = x.shape
    g = x.reshape(B, C // 32, 32, H, W)
    amax = g.abs().amax(dim=2, keepdim=True).clamp_min(1e-30)
    s = torch.pow(2.0, torch.ceil(torch.log2(amax / 448.0)))
    return ((g / s).clamp(-448, 448).to(torch.float8_e4m3fn).float() * s).reshape(B, C, H, W)
groups = {"l3 16-29": [f"layer3.{i}.conv{c}" for i in range(16, 30) for c in (1, 2)],
          "l3 1-29": [f"layer3.{i}.conv{c}" for i in range(1, 30) for c in (1, 2)],
          "l2+l3 stages": [f"layer3.{i}.conv{c}" for i in range(1, 30) for c in (1, 2)] + [f"layer2.{i}.conv{c}" for i in range(1, 13) for c in (1, 2)]}
for mode in ("image", "mx32"):
    if mode == "mx32": P.q_act = q_mx
    for g, mem in groups.items():
        e = P.cos_err(model, xin, ref, set(mem))
        print(mode, g, f"mean {e.mean():.2e} max {e.max():.2e}", flush=True)
