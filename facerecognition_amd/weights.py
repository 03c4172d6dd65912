"""Weights: reference checkpoint schema → BN-folded FRW1 blob for libfrhip; synthetic weights.

* ``param_specs(arch)`` lists every state_dict entry of the three backbones with the exact
  key names the reference (or its external modules) uses:
  - ``resnet50_arcface``: ``ArcFaceModel`` (models/arcface/arcface_model.py:135-202) with the
    torchvision ResNet-50 trunk copied at :88-98 (keys ``backbone.*``, ``bn1``, ``fc``, ``bn2``,
    ``arcface.weight``).
  - ``iresnet100``: insightface ``iresnet100`` (IBasicBlock; README.md:72 names it, no code).
  - ``irv1_facenet``: ``FaceNetModel`` (models/facenet/facenet_model.py:7-36) wrapping
    facenet-pytorch ``InceptionResnetV1`` (keys ``model.*``, optional ``projection``).
* ``synth_state_dict`` fills those entries from a counter-based splitmix64 stream (seeded,
  platform independent, no torch RNG) plus BN running statistics calibrated once on random
  crops (``facerecognition_amd/synth/<arch>_bnstats.npz``, written by tools/calibrate_bn.py);
  SURVEY.md §0.5 explains why uncalibrated random BN stats collapse the embeddings.
* ``fold_state_dict`` folds every eval-mode BatchNorm into the adjacent conv/linear (in f64)
  and emits the tensor names the native plans in csrc/engine.cpp expect.
* ``load_checkpoint`` reads the reference's training checkpoint schema
  (``model_state_dict``/``config``/``num_classes``; models/arcface/train_arcface.py:755-772)
  with ``torch.load(weights_only=True)`` — never an unpickling loader.
"""
from __future__ import annotations

import io
import os
import struct
from typing import Dict, List, Optional, Tuple

import numpy as np

ARCHS = ("resnet50_arcface", "iresnet100", "irv1_facenet")
# Default compute dtype per backbone: bf16 as BASELINE.json names it (configs 2-3).  The
# bf16 InceptionResnetV1 plan stores and multiplies its high-resolution stem (conv2d_1a .. conv2d_4a) in
# f16: all-bf16 missed the 1e-3 cosine bar (~2e-3, the stem's rounding dominates; tools/drift_compare.py).
DEFAULT_DTYPE = {"resnet50_arcface": "bf16", "iresnet100": "bf16", "irv1_facenet": "bf16"}
ARCH_IDS = {"resnet50_arcface": 0, "iresnet100": 1, "irv1_facenet": 2}
INPUT_SIZE = {"resnet50_arcface": 112, "iresnet100": 112, "irv1_facenet": 160}
BN_EPS = {"resnet50_arcface": 1e-5, "iresnet100": 1e-5, "irv1_facenet": 1e-3}
SYNTH_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "synth")

Spec = Tuple[str, Tuple[int, ...], str]  # (key, shape, kind)


# ----------------------------------------------------------------------------- specs
def _bn(p: str, c: int) -> List[Spec]:
    return [(p + ".weight", (c,), "bn_w"), (p + ".bias", (c,), "bn_b"),
            (p + ".running_mean", (c,), "bn_rm"), (p + ".running_var", (c,), "bn_rv"),
            (p + ".num_batches_tracked", (), "nbt")]


def _conv(p: str, cout: int, cin: int, kh: int, kw: int) -> List[Spec]:
    return [(p + ".weight", (cout, cin, kh, kw), "conv")]


def _specs_resnet50(num_classes: int = 100, emb: int = 512) -> List[Spec]:
    s = _conv("backbone.conv1", 64, 3, 7, 7) + _bn("backbone.bn1", 64)
    inpl = 64
    for li, (planes, blocks) in enumerate([(64, 3), (128, 4), (256, 6), (512, 3)]):
        for i in range(blocks):
            p = f"backbone.layer{li + 1}.{i}"
            s += _conv(p + ".conv1", planes, inpl, 1, 1) + _bn(p + ".bn1", planes)
            s += _conv(p + ".conv2", planes, planes, 3, 3) + _bn(p + ".bn2", planes)
            s += _conv(p + ".conv3", planes * 4, planes, 1, 1) + _bn(p + ".bn3", planes * 4)
            if i == 0:
                s += _conv(p + ".downsample.0", planes * 4, inpl, 1, 1) + _bn(p + ".downsample.1", planes * 4)
            inpl = planes * 4
    s += _bn("bn1", 2048)
    s += [("fc.weight", (emb, 2048), "linear"), ("fc.bias", (emb,), "bias")]
    s += _bn("bn2", emb)
    s += [("arcface.weight", (num_classes, emb), "arc")]
    return s


def _specs_iresnet100() -> List[Spec]:
    s = _conv("conv1", 64, 3, 3, 3) + _bn("bn1", 64) + [("prelu.weight", (64,), "prelu")]
    inpl = 64
    for li, (planes, blocks) in enumerate([(64, 3), (128, 13), (256, 30), (512, 3)]):
        for i in range(blocks):
            p = f"layer{li + 1}.{i}"
            s += _bn(p + ".bn1", inpl)
            s += _conv(p + ".conv1", planes, inpl, 3, 3) + _bn(p + ".bn2", planes)
            s += [(p + ".prelu.weight", (planes,), "prelu")]
            s += _conv(p + ".conv2", planes, planes, 3, 3) + _bn(p + ".bn3", planes)
            if i == 0:
                s += _conv(p + ".downsample.0", planes, inpl, 1, 1) + _bn(p + ".downsample.1", planes)
            inpl = planes
    s += _bn("bn2", 512)
    s += [("fc.weight", (512, 512 * 49), "linear"), ("fc.bias", (512,), "bias")]
    s += _bn("features", 512)
    return s


def _basic(p: str, cin: int, cout: int, kh: int, kw: int) -> List[Spec]:
    return _conv(p + ".conv", cout, cin, kh, kw) + _bn(p + ".bn", cout)


def _specs_irv1(emb: int = 512) -> List[Spec]:
    m = "model."
    s = _basic(m + "conv2d_1a", 3, 32, 3, 3) + _basic(m + "conv2d_2a", 32, 32, 3, 3)
    s += _basic(m + "conv2d_2b", 32, 64, 3, 3) + _basic(m + "conv2d_3b", 64, 80, 1, 1)
    s += _basic(m + "conv2d_4a", 80, 192, 3, 3) + _basic(m + "conv2d_4b", 192, 256, 3, 3)
    for i in range(5):
        p = f"{m}repeat_1.{i}."
        s += _basic(p + "branch0", 256, 32, 1, 1)
        s += _basic(p + "branch1.0", 256, 32, 1, 1) + _basic(p + "branch1.1", 32, 32, 3, 3)
        s += _basic(p + "branch2.0", 256, 32, 1, 1) + _basic(p + "branch2.1", 32, 32, 3, 3)
        s += _basic(p + "branch2.2", 32, 32, 3, 3)
        s += [(p + "conv2d.weight", (256, 96, 1, 1), "conv"), (p + "conv2d.bias", (256,), "bias")]
    p = m + "mixed_6a."
    s += _basic(p + "branch0", 256, 384, 3, 3)
    s += _basic(p + "branch1.0", 256, 192, 1, 1) + _basic(p + "branch1.1", 192, 192, 3, 3)
    s += _basic(p + "branch1.2", 192, 256, 3, 3)
    for i in range(10):
        p = f"{m}repeat_2.{i}."
        s += _basic(p + "branch0", 896, 128, 1, 1)
        s += _basic(p + "branch1.0", 896, 128, 1, 1) + _basic(p + "branch1.1", 128, 128, 1, 7)
        s += _basic(p + "branch1.2", 128, 128, 7, 1)
        s += [(p + "conv2d.weight", (896, 256, 1, 1), "conv"), (p + "conv2d.bias", (896,), "bias")]
    p = m + "mixed_7a."
    s += _basic(p + "branch0.0", 896, 256, 1, 1) + _basic(p + "branch0.1", 256, 384, 3, 3)
    s += _basic(p + "branch1.0", 896, 256, 1, 1) + _basic(p + "branch1.1", 256, 256, 3, 3)
    s += _basic(p + "branch2.0", 896, 256, 1, 1) + _basic(p + "branch2.1", 256, 256, 3, 3)
    s += _basic(p + "branch2.2", 256, 256, 3, 3)
    for i in range(6):
        p = f"{m}repeat_3.{i}." if i < 5 else m + "block8."
        s += _basic(p + "branch0", 1792, 192, 1, 1)
        s += _basic(p + "branch1.0", 1792, 192, 1, 1) + _basic(p + "branch1.1", 192, 192, 1, 3)
        s += _basic(p + "branch1.2", 192, 192, 3, 1)
        s += [(p + "conv2d.weight", (1792, 384, 1, 1), "conv"), (p + "conv2d.bias", (1792,), "bias")]
    s += [(m + "last_linear.weight", (512, 1792), "linear")] + _bn(m + "last_bn", 512)
    if emb != 512:
        s += [("projection.weight", (emb, 512), "linear"), ("projection.bias", (emb,), "bias")]
    return s


def param_specs(arch: str, num_classes: int = 100, embedding_size: int = 512) -> List[Spec]:
    if arch == "resnet50_arcface":
        return _specs_resnet50(num_classes, embedding_size)
    if arch == "iresnet100":
        return _specs_iresnet100()
    if arch == "irv1_facenet":
        return _specs_irv1(embedding_size)
    raise ValueError(f"unknown arch {arch!r}; expected one of {ARCHS}")


# ----------------------------------------------------------------------------- synthetic
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for ch in s.encode():
        h ^= ch
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def splitmix_uniform(seed: int, name: str, n: int) -> np.ndarray:
    """Uniform [0,1) float64 stream: splitmix64((seed ^ fnv1a64(name)) + i*golden)."""
    with np.errstate(over="ignore"):
        base = np.uint64((seed ^ _fnv1a64(name)) & 0xFFFFFFFFFFFFFFFF)
        z = base + (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def _synth_value(seed: int, key: str, shape: Tuple[int, ...], kind: str) -> np.ndarray:
    n = int(np.prod(shape)) if shape else 1
    if kind == "nbt":
        return np.array(1, dtype=np.int64)
    if kind == "bn_rm":
        return np.zeros(shape, np.float32)
    if kind == "bn_rv":
        return np.ones(shape, np.float32)
    u = splitmix_uniform(seed, key, n)
    if kind == "conv":
        fan_in = shape[1] * shape[2] * shape[3]
        v = (2 * u - 1) * np.sqrt(6.0 / fan_in)
    elif kind == "linear":
        v = (2 * u - 1) * np.sqrt(3.0 / shape[1])
    elif kind == "bn_w" and key.endswith("bn3.weight"):
        # last BN of a residual branch (ResNet Bottleneck / IBasicBlock): small gain, the
        # 'zero-init-residual' convention, so the synthetic trunk is not chaotic
        v = 0.1 + 0.2 * u
    elif kind == "bn_w":
        v = 1.0 + 0.2 * (u - 0.5)
    elif kind in ("bn_b", "bias"):
        v = 0.2 * (u - 0.5)
    elif kind == "prelu":
        v = 0.25 + 0.1 * (u - 0.5)
    elif kind == "arc":
        v = u - 0.5
    else:
        raise ValueError(kind)
    return v.astype(np.float32).reshape(shape)


def bnstats_path(arch: str) -> str:
    return os.path.join(SYNTH_DIR, f"{arch}_bnstats.npz")


def synth_state_dict(arch: str, seed: int = 1234, calibrated: bool = True, num_classes: int = 100,
                     embedding_size: int = 512) -> Dict[str, np.ndarray]:
    """Deterministic synthetic state_dict in the reference key schema."""
    sd = {k: _synth_value(seed, k, shp, kind)
          for k, shp, kind in param_specs(arch, num_classes, embedding_size)}
    if calibrated:
        path = bnstats_path(arch)
        if not os.path.exists(path):
            raise FileNotFoundError(f"BN calibration stats missing: {path} (run tools/calibrate_bn.py)")
        with np.load(path, allow_pickle=False) as z:
            if int(z["__seed__"]) != seed:
                raise ValueError(f"{path} was calibrated for seed {int(z['__seed__'])}, not {seed}")
            for k in z.files:
                if k.startswith("__"):
                    continue
                if k not in sd or sd[k].shape != z[k].shape:
                    raise ValueError(f"calibration entry {k} does not match the {arch} spec")
                sd[k] = z[k].astype(np.float32)
    return sd


# ----------------------------------------------------------------------------- folding
def _np(x) -> np.ndarray:
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def _bn_affine(sd, p: str, eps: float) -> Tuple[np.ndarray, np.ndarray]:
    g = _np(sd[p + ".weight"]).astype(np.float64)
    b = _np(sd[p + ".bias"]).astype(np.float64)
    rm = _np(sd[p + ".running_mean"]).astype(np.float64)
    rv = _np(sd[p + ".running_var"]).astype(np.float64)
    s = g / np.sqrt(rv + eps)
    return s, b - rm * s


def _krsc(w) -> np.ndarray:
    return np.ascontiguousarray(_np(w).astype(np.float64).transpose(0, 2, 3, 1))


def _put_conv(out: dict, name: str, w: np.ndarray, s: Optional[np.ndarray], t: Optional[np.ndarray],
              slope=None) -> None:
    w = w if s is None else w * s[:, None, None, None]
    out[name + ".w"] = w.astype(np.float32)
    out[name + ".b"] = (t if t is not None else np.zeros(w.shape[0])).astype(np.float32)
    if slope is not None:
        out[name + ".slope"] = _np(slope).astype(np.float32)


def _fold_pre_bn_3x3(out: dict, name: str, w: np.ndarray, s1, t1, s2, t2, slope) -> None:
    """IBasicBlock conv1 with its PRE-conv BN folded in: bn2(conv(pad0(s1*x + t1))).

    Zero padding is applied after bn1, so its shift t1 only reaches the taps that land inside the image:
        conv(pad0(s1*x + t1), W) = conv(pad0(x), W*s1) + sum_{taps inside} sum_c W[o,c,tap] t1[c].
    The second term depends only on the output pixel's border class (top / interior / bottom row x left /
    interior / right column for 3x3, stride 1, pad 1), so it becomes a [9, Cout] bias table '.b9'
    (class 3*rc + cc).  bn2 folds into the output side as usual.  w: [Cout, 3, 3, Cin] (KRSC), f64."""
    ws = w * s2[:, None, None, None]                       # bn2 (output side)
    T = np.einsum("orsc,c->ors", ws, t1)                   # bn1 shift through each tap: [Cout, 3, 3]
    valid = ((1, 2), (0, 1, 2), (0, 1))                    # taps inside the image for rc / cc = 0, 1, 2
    b9 = np.stack([t2 + T[:, list(valid[rc]), :][:, :, list(valid[cc])].sum(axis=(1, 2))
                   for rc in range(3) for cc in range(3)])
    out[name + ".w"] = (ws * s1[None, None, None, :]).astype(np.float32)
    out[name + ".b"] = b9[4].astype(np.float32)            # interior class (reference only)
    out[name + ".b9"] = b9.astype(np.float32)
    out[name + ".slope"] = _np(slope).astype(np.float32)


def fold_state_dict(arch: str, sd) -> Dict[str, np.ndarray]:
    """Eval-mode BN folding (f64) → the tensor names of csrc/engine.cpp's plans."""
    eps = BN_EPS[arch]
    out: Dict[str, np.ndarray] = {}
    if arch == "resnet50_arcface":
        s, t = _bn_affine(sd, "backbone.bn1", eps)
        _put_conv(out, "backbone.conv1", _krsc(sd["backbone.conv1.weight"]), s, t)
        for li, blocks in enumerate([3, 4, 6, 3]):
            for i in range(blocks):
                p = f"backbone.layer{li + 1}.{i}"
                for c, bn in (("conv1", "bn1"), ("conv2", "bn2"), ("conv3", "bn3")):
                    s, t = _bn_affine(sd, f"{p}.{bn}", eps)
                    _put_conv(out, f"{p}.{c}", _krsc(sd[f"{p}.{c}.weight"]), s, t)
                if i == 0:
                    s, t = _bn_affine(sd, f"{p}.downsample.1", eps)
                    _put_conv(out, f"{p}.downsample", _krsc(sd[f"{p}.downsample.0.weight"]), s, t)
        # head: bn2(fc(dropout(bn1(x)))) — arcface_model.py:192-196; dropout is identity in eval.
        s1, t1 = _bn_affine(sd, "bn1", eps)
        s2, t2 = _bn_affine(sd, "bn2", eps)
        W = _np(sd["fc.weight"]).astype(np.float64)
        bfc = _np(sd["fc.bias"]).astype(np.float64)
        out["head.w"] = (s2[:, None] * W * s1[None, :]).astype(np.float32)
        out["head.b"] = (s2 * (W @ t1 + bfc) + t2).astype(np.float32)
    elif arch == "iresnet100":
        s, t = _bn_affine(sd, "bn1", eps)
        _put_conv(out, "conv1", _krsc(sd["conv1.weight"]), s, t, sd["prelu.weight"])
        for li, blocks in enumerate([3, 13, 30, 3]):
            for i in range(blocks):
                p = f"layer{li + 1}.{i}"
                s1, t1 = _bn_affine(sd, p + ".bn1", eps)
                s2, t2 = _bn_affine(sd, p + ".bn2", eps)
                _fold_pre_bn_3x3(out, p + ".conv1", _krsc(sd[p + ".conv1.weight"]), s1, t1, s2, t2,
                                 sd[p + ".prelu.weight"])
                s, t = _bn_affine(sd, p + ".bn3", eps)
                _put_conv(out, p + ".conv2", _krsc(sd[p + ".conv2.weight"]), s, t)
                if i == 0:
                    s, t = _bn_affine(sd, p + ".downsample.1", eps)
                    _put_conv(out, p + ".downsample", _krsc(sd[p + ".downsample.0.weight"]), s, t)
        # head: features(fc(flatten(bn2(x)))); torch flattens NCHW (c*49 + p), we read NHWC (p*512 + c).
        s2, t2 = _bn_affine(sd, "bn2", eps)
        sf, tf = _bn_affine(sd, "features", eps)
        W = _np(sd["fc.weight"]).astype(np.float64).reshape(512, 512, 49)  # [o][c][p]
        bfc = _np(sd["fc.bias"]).astype(np.float64)
        Wn = (W * s2[None, :, None]).transpose(0, 2, 1).reshape(512, 49 * 512)  # [o][p*512+c]
        out["head.w"] = (sf[:, None] * Wn).astype(np.float32)
        out["head.b"] = (sf * (bfc + np.einsum("ocp,c->o", W, t2)) + tf).astype(np.float32)
    elif arch == "irv1_facenet":
        m = "model."

        def basic(p):
            s, t = _bn_affine(sd, p + ".bn", eps)
            _put_conv(out, p, _krsc(sd[p + ".conv.weight"]), s, t)

        for n in ("conv2d_1a", "conv2d_2a", "conv2d_2b", "conv2d_3b", "conv2d_4a", "conv2d_4b"):
            basic(m + n)

        def block(p, branches, scale):
            for b in branches:
                basic(p + b)
            w = _krsc(sd[p + "conv2d.weight"]) * scale  # out = conv2d(cat)*scale + x
            out[p + "conv2d.w"] = w.astype(np.float32)
            out[p + "conv2d.b"] = (_np(sd[p + "conv2d.bias"]).astype(np.float64) * scale).astype(np.float32)

        for i in range(5):
            block(f"{m}repeat_1.{i}.", ["branch0", "branch1.0", "branch1.1", "branch2.0", "branch2.1",
                                       "branch2.2"], 0.17)
        for b in ("branch0", "branch1.0", "branch1.1", "branch1.2"):
            basic(m + "mixed_6a." + b)
        for i in range(10):
            block(f"{m}repeat_2.{i}.", ["branch0", "branch1.0", "branch1.1", "branch1.2"], 0.10)
        for b in ("branch0.0", "branch0.1", "branch1.0", "branch1.1", "branch2.0", "branch2.1", "branch2.2"):
            basic(m + "mixed_7a." + b)
        for i in range(6):
            p = f"{m}repeat_3.{i}." if i < 5 else m + "block8."
            block(p, ["branch0", "branch1.0", "branch1.1", "branch1.2"], 0.20 if i < 5 else 1.0)
        sl, tl = _bn_affine(sd, m + "last_bn", eps)
        W = _np(sd[m + "last_linear.weight"]).astype(np.float64)
        out["head.w"] = (sl[:, None] * W).astype(np.float32)
        out["head.b"] = tl.astype(np.float32)
        if "projection.weight" in sd:  # FaceNetModel.projection (facenet_model.py:20-23,32-33), after IRV1's L2
            out["proj.w"] = _np(sd["projection.weight"]).astype(np.float32)
            out["proj.b"] = _np(sd["projection.bias"]).astype(np.float32)
    else:
        raise ValueError(arch)
    return out


# Mixed fp8 / bf16 plans (BASELINE config 5): the convs that run in e4m3.  IResNet100: the tail of layer3
# (blocks 16..29, conv1 + conv2: 28 convs, 28 % of the FLOPs), the least sensitive convs of the per-conv
# sweep in profiles/r03_fp8_plan.json (tools/fp8_plan.py: together 1 - cos ~6e-4 against fp32, under
# the 1e-3 bar; all of layer3 measures 1.6e-3, every conv 8.6e-3).  They run as one e4m3 LDS-resident
# stage (conv_stage8.hip).  Other archs: no plan measured, every eligible conv.
FP8_PLAN = {
    "iresnet100": tuple(f"layer3.{i}.conv{j}" for i in range(16, 30) for j in (1, 2)),
}


def fp8_plan(arch: str):
    """The conv names FR_DTYPE_FP8 quantizes for `arch` (None = every eligible conv).  FR_FP8_PLAN=all
    overrides the plan (every eligible conv; A/B only)."""
    if os.environ.get("FR_FP8_PLAN") == "all":
        return None
    return FP8_PLAN.get(arch)


def quantize_fp8(folded: Dict[str, np.ndarray], min_cin: int = 64, convs=None) -> Dict[str, np.ndarray]:
    """FR_DTYPE_FP8 weights (BASELINE config 5): the folded conv weights "<name>.w" [Cout, kh, kw, Cin]
    with Cin % 64 == 0 -- those named in `convs`, or every one when None -- become per-output-channel
    scaled OCP e4m3: s[o] = max|w[o]| / 448 (f32), "<name>.w" = e4m3(w / s) as exactly representable f32
    values (torch.float8_e4m3fn cast, RNE, saturating), "<name>.wscale" = s.  The stem (Cin 3) and the
    2-D head stay bf16.  Dequantized weight = w * s.  Biases, border-class tables and PReLU slopes are
    unchanged; convs without a .wscale run in bf16."""
    import torch
    out = dict(folded)
    want = None if convs is None else set(convs)
    for k, w in folded.items():
        if not k.endswith(".w") or w.ndim != 4 or w.shape[3] % min_cin != 0:
            continue
        if want is not None and k[:-2] not in want:
            continue
        w64 = np.asarray(w, dtype=np.float32)
        amax = np.abs(w64).reshape(w64.shape[0], -1).max(axis=1)
        s = np.where(amax > 0, amax / 448.0, 1.0).astype(np.float32)
        q = torch.from_numpy(w64 / s[:, None, None, None]).clamp(-448, 448).to(torch.float8_e4m3fn)
        out[k] = q.to(torch.float32).numpy()
        out[k[:-2] + ".wscale"] = s
    return out


def pack_blob(tensors: Dict[str, np.ndarray]) -> bytes:
    """FRW1 := "FRW1" u32 count { u32 len, name, u32 ndim, i64 dims[], f32 data[] }*"""
    buf = io.BytesIO()
    buf.write(b"FRW1")
    buf.write(struct.pack("<I", len(tensors)))
    for name, arr in tensors.items():
        a = np.ascontiguousarray(np.asarray(arr, dtype=np.float32))
        nb = name.encode()
        buf.write(struct.pack("<I", len(nb)))
        buf.write(nb)
        buf.write(struct.pack("<I", a.ndim))
        buf.write(struct.pack("<%dq" % a.ndim, *a.shape))
        buf.write(a.tobytes())
    return buf.getvalue()


# ----------------------------------------------------------------------------- checkpoints
def detect_arch(sd) -> str:
    keys = set(sd.keys())
    if "backbone.conv1.weight" in keys:
        return "resnet50_arcface"
    if "model.conv2d_1a.conv.weight" in keys or "conv2d_1a.conv.weight" in keys:
        return "irv1_facenet"
    if "conv1.weight" in keys and "layer3.29.conv2.weight" in keys:
        return "iresnet100"
    raise ValueError("unrecognised state_dict: not ResNet-50 ArcFace, IResNet100 or InceptionResnetV1")


def load_checkpoint(path: str) -> Tuple[dict, dict]:
    """Read a reference training checkpoint (train_arcface.py:755-772) without unpickling code."""
    import torch
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(ck, dict) and "model_state_dict" in ck:
        sd = ck["model_state_dict"]
    elif isinstance(ck, dict) and "state_dict" in ck:
        sd = ck["state_dict"]
    else:
        sd = ck
    sd = {k: v for k, v in sd.items()}
    # FaceNet checkpoints may store the trunk without the 'model.' prefix, or with a
    # 'backbone.' prefix, and carry unused 'logits.*' (models/facenet/checkpoint_utils.py:5-110).
    if "conv2d_1a.conv.weight" in sd or "backbone.conv2d_1a.conv.weight" in sd:
        re = {}
        for k, v in sd.items():
            if k.startswith("logits.") or k.startswith("model.logits.") or k.startswith("backbone.logits."):
                continue
            if k.startswith("backbone."):
                k = "model." + k[len("backbone."):]
            elif not k.startswith("model.") and not k.startswith("projection."):
                k = "model." + k
            re[k] = v
        sd = re
    info = {k: ck.get(k) for k in ("num_classes", "epoch", "best_val_acc", "val_acc")} if isinstance(ck, dict) else {}
    info["config"] = ck.get("config", {}) if isinstance(ck, dict) else {}
    return sd, info
