#!/usr/bin/env python3
"""Per-conv fp8 sensitivity of IResNet100 and the mixed fp8/bf16 plan for BASELINE config 5 (CPU only).

The fp32 oracle (oracle/models.py) is run with ONE conv at a time fake-quantized the way the GPU fp8
path computes it -- weights as folded by weights.fold_state_dict (the pre-conv bn1 scale multiplied into
conv1's input channels; bn2 / bn3 / downsample BN are per-output-channel factors, which commute with the
per-output-channel e4m3 quantizer) in OCP e4m3 with a per-output-channel scale, and the conv's input
activation in e4m3 with a power-of-two scale from its amax (per image: the stage kernel's scale; the
border-class bias of the folded bn1 shift stays exact).  Each conv's 1 - cos against the unquantized
oracle is its sensitivity; sets of convs are then measured together.

    python tools/fp8_plan.py [--n 8] [--out profiles/r03_fp8_plan.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def q_w(w):
    """Per-output-channel e4m3 (weights.quantize_fp8's quantizer)."""
    amax = w.abs().reshape(w.shape[0], -1).amax(dim=1)
    s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax)).view(-1, 1, 1, 1)
    return (w / s).clamp(-448, 448).to(torch.float8_e4m3fn).float() * s


def q_act(x):
    """e4m3 with a power-of-two scale per image: 2^e, the smallest with amax / 2^e <= 448."""
    amax = x.abs().reshape(x.shape[0], -1).amax(dim=1).clamp_min(1e-30)
    e = torch.ceil(torch.log2(amax / 448.0))
    s = torch.pow(2.0, e).view(-1, 1, 1, 1)
    return (x / s).clamp(-448, 448).to(torch.float8_e4m3fn).float() * s


def bn_affine(bn):
    a = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    return a, bn.bias - bn.running_mean * a


def conv_names(model):
    out = []
    for l in range(1, 5):
        for i, blk in enumerate(getattr(model, f"layer{l}")):
            out += [f"layer{l}.{i}.conv1", f"layer{l}.{i}.conv2"]
            if blk.downsample is not None:
                out.append(f"layer{l}.{i}.downsample")
    return out


def conv_flops(model):
    """Algorithmic FLOPs per face of every conv (112x112 input)."""
    fl, hooks = {}, []
    for name, m in model.named_modules():
        if isinstance(m, torch.nn.Conv2d):
            def h(mod, inp, out, name=name):
                fl[name[:-2] if name.endswith("downsample.0") else name] = \
                    2.0 * out.shape[2] * out.shape[3] * mod.out_channels * mod.in_channels * mod.kernel_size[0] * mod.kernel_size[1]
            hooks.append(m.register_forward_hook(h))
    with torch.no_grad():
        model(torch.zeros(1, 3, 112, 112))
    for h in hooks:
        h.remove()
    return fl


def forward_q(model, x, qset):
    """IResNet100 forward with the convs in qset fake-quantized (weights + input activation)."""
    x = model.prelu(model.bn1(model.conv1(x)))
    for l in range(1, 5):
        for i, blk in enumerate(getattr(model, f"layer{l}")):
            p = f"layer{l}.{i}."
            idt = x
            if p + "conv1" in qset:  # conv1(pad(bn1(x))) = conv(pad(a x), w) + conv(pad(b 1), w)
                a, b = bn_affine(blk.bn1)
                wf = q_w(blk.conv1.weight * a.view(1, -1, 1, 1))
                out = F.conv2d(q_act(x), wf, padding=1) + F.conv2d(b.view(1, -1, 1, 1).expand_as(x), blk.conv1.weight, padding=1)
            else:
                out = blk.conv1(blk.bn1(x))
            out = blk.prelu(blk.bn2(out))
            w2 = q_w(blk.conv2.weight) if p + "conv2" in qset else blk.conv2.weight
            o2 = F.conv2d(q_act(out) if p + "conv2" in qset else out, w2, stride=blk.conv2.stride, padding=1)
            out = blk.bn3(o2)
            if blk.downsample is not None:
                ds = blk.downsample[0]
                if p + "downsample" in qset:
                    idt = blk.downsample[1](F.conv2d(q_act(x), q_w(ds.weight), stride=ds.stride))
                else:
                    idt = blk.downsample(x)
            x = out + idt
    x = torch.flatten(model.bn2(x), 1)
    return F.normalize(model.features(model.fc(x)), dim=1)


def cos_err(model, xin, ref, qset):
    with torch.no_grad():
        e = forward_q(model, xin, qset)
    return (1 - (e * ref).sum(1)).numpy()


def main():
    from facerecognition_amd.synthetic import synthetic_crops
    from facerecognition_amd.weights import synth_state_dict
    from oracle import models as M
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--budget", type=float, default=6e-4, help="mean 1-cos budget of the chosen fp8 set")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    model = M.build_model("iresnet100", synth_state_dict("iresnet100")).eval()
    xin = M.preprocess_u8_nhwc(synthetic_crops(a.n, 112, seed=4))
    with torch.no_grad():
        ref = forward_q(model, xin, set())
        ref0 = F.normalize(model(xin), dim=1)
    assert float((ref - ref0).abs().max()) < 1e-5, "forward_q restates the oracle forward"
    names = conv_names(model)
    fl = conv_flops(model)
    total = sum(fl.values()) + 2.0 * 512 * 25088
    t0 = time.time()
    sens = {}
    for nm in names:
        sens[nm] = float(cos_err(model, xin, ref, {nm}).mean())
    print(f"per-conv sensitivity ({len(names)} convs, {time.time() - t0:.0f}s)")
    for nm in names:
        print(f"  {nm:24s} {sens[nm]:.2e}  {fl[nm] / 1e9:.3f} GFLOP/face")
    groups = {
        "layer3 stage (layer3.1-29 conv1+conv2)": [f"layer3.{i}.conv{c}" for i in range(1, 30) for c in (1, 2)],
        "layer2 stage (layer2.1-12)": [f"layer2.{i}.conv{c}" for i in range(1, 13) for c in (1, 2)],
        "layer1 stage (layer1.1-2)": [f"layer1.{i}.conv{c}" for i in range(1, 3) for c in (1, 2)],
        "layer4 (all)": [n for n in names if n.startswith("layer4")],
        "all convs": names,
    }
    res = {"n_faces": a.n, "sensitivity": sens, "gflop_per_face": {k: fl[k] / 1e9 for k in names}, "groups": {}}
    for g, members in groups.items():
        e = cos_err(model, xin, ref, set(members))
        frac = sum(fl[m] for m in members) / total
        res["groups"][g] = {"mean": float(e.mean()), "max": float(e.max()), "flop_frac": frac}
        print(f"{g:42s} 1-cos mean {e.mean():.2e} max {e.max():.2e}   {100 * frac:.1f} % of FLOPs")
    # greedy plan: least sensitivity per FLOP first, while the measured set stays within budget
    order = sorted(names, key=lambda n: sens[n] / fl[n])
    chosen, cur = [], 0.0
    for nm in order:
        if cur + sens[nm] > a.budget:
            continue
        chosen.append(nm)
        cur += sens[nm]
    e = cos_err(model, xin, ref, set(chosen))
    frac = sum(fl[m] for m in chosen) / total
    print(f"greedy set: {len(chosen)} convs, {100 * frac:.1f} % of FLOPs, predicted {cur:.2e}, measured mean "
          f"{e.mean():.2e} max {e.max():.2e}")
    res["greedy"] = {"convs": chosen, "flop_frac": frac, "mean": float(e.mean()), "max": float(e.max())}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
