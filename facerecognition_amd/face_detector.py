"""Face detection before the embedding path on the MI355X.

The reference detects faces with facenet-pytorch's MTCNN behind ``FaceDetector`` (preprocessing/
face_detector.py:78-97 ``MTCNN(image_size=160, margin=0, min_face_size=20, thresholds=[0.6, 0.7, 0.7],
factor=0.709, post_process=False, keep_all=True)``; ``_detect_mtcnn`` :144-210) and aligns the chosen face
to ``ARCFACE_TEMPLATE`` (inference/recognition_engine.py:169-242).  Here the P/R/O-nets, the image pyramid
and the box crops run on the device through libfrhip.so (mtcnn.hip: f32 area resampling bit-identical to
torch, f32 convs / pools / dense layers / heads); the per-stage box bookkeeping -- thresholding,
non-maximum suppression, box regression, squaring and padding, a few hundred boxes -- is host logic, as
in the reference, whose last NMS is numpy as well (``detect_face``'s ``batched_nms_numpy``).  The
alignment warp is ``align.align_faces`` (device, OpenCV's fixed-point warpAffine).

Weights: facenet-pytorch's pretrained pnet.pt / rnet.pt / onet.pt are not in the reference or this
image.  ``load_mtcnn_state(dir)`` reads them when supplied (state dicts, ``torch.load(weights_only=True)``);
``synth_mtcnn_state`` makes seeded synthetic ones (test parity against oracle/mtcnn.py only: their
detections mean nothing).  Without weights the detector is unavailable, exactly like the reference
without facenet-pytorch (RecognitionEngine then runs on the raw image).
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N

THRESHOLDS = (0.6, 0.7, 0.7)
FACTOR = 0.709
MIN_FACE = 20
# synth_mtcnn_state: face-classification head gains and (background, face) logit offsets
HEAD_GAIN = {"conv4_1": 40.0, "dense5_1": 40.0, "dense6_1": 150.0}
SYNTH_LOGIT_SHIFT = {"rnet.dense5_1.bias": (-0.6, 0.6)}
# synth_mtcnn_state(calibrated=True): extra (face - background) logit offsets measured by tools/calibrate_mtcnn.py
# so that, on tools/mtcnn_bench.py's 1080p frame, P-net passes ~1 % of its windows, R-net ~10 % and O-net ~30 % of
# their inputs -- the box volumes of a trained detector on a frame with a few faces (assumed; the stress weights
# above pass 92 % of P-net windows and carry 10^5 boxes through every stage)
CALIBRATED_LOGIT_SHIFT = {"pnet.conv4_1.bias": 2.34, "rnet.dense5_1.bias": 0.29, "onet.dense6_1.bias": 7.04}
LANDMARK_NAMES = ("left_eye", "right_eye", "nose", "left_mouth", "right_mouth")

# facenet-pytorch's P/R/O-net parameters (name -> shape), models/mtcnn.py
MTCNN_SPECS = {
    "pnet": [("conv1.weight", (10, 3, 3, 3)), ("conv1.bias", (10,)), ("prelu1.weight", (10,)),
             ("conv2.weight", (16, 10, 3, 3)), ("conv2.bias", (16,)), ("prelu2.weight", (16,)),
             ("conv3.weight", (32, 16, 3, 3)), ("conv3.bias", (32,)), ("prelu3.weight", (32,)),
             ("conv4_1.weight", (2, 32, 1, 1)), ("conv4_1.bias", (2,)),
             ("conv4_2.weight", (4, 32, 1, 1)), ("conv4_2.bias", (4,))],
    "rnet": [("conv1.weight", (28, 3, 3, 3)), ("conv1.bias", (28,)), ("prelu1.weight", (28,)),
             ("conv2.weight", (48, 28, 3, 3)), ("conv2.bias", (48,)), ("prelu2.weight", (48,)),
             ("conv3.weight", (64, 48, 2, 2)), ("conv3.bias", (64,)), ("prelu3.weight", (64,)),
             ("dense4.weight", (128, 576)), ("dense4.bias", (128,)), ("prelu4.weight", (128,)),
             ("dense5_1.weight", (2, 128)), ("dense5_1.bias", (2,)),
             ("dense5_2.weight", (4, 128)), ("dense5_2.bias", (4,))],
    "onet": [("conv1.weight", (32, 3, 3, 3)), ("conv1.bias", (32,)), ("prelu1.weight", (32,)),
             ("conv2.weight", (64, 32, 3, 3)), ("conv2.bias", (64,)), ("prelu2.weight", (64,)),
             ("conv3.weight", (64, 64, 3, 3)), ("conv3.bias", (64,)), ("prelu3.weight", (64,)),
             ("conv4.weight", (128, 64, 2, 2)), ("conv4.bias", (128,)), ("prelu4.weight", (128,)),
             ("dense5.weight", (256, 1152)), ("dense5.bias", (256,)), ("prelu5.weight", (256,)),
             ("dense6_1.weight", (2, 256)), ("dense6_1.bias", (2,)),
             ("dense6_2.weight", (4, 256)), ("dense6_2.bias", (4,)),
             ("dense6_3.weight", (10, 256)), ("dense6_3.bias", (10,))],
}


def synth_mtcnn_state(seed: int = 7, calibrated: bool = False) -> Dict[str, np.ndarray]:
    """Seeded synthetic P/R/O-net weights (the splitmix stream of weights.synth_state_dict): layers with
    torch's default uniform init bound, PReLU 0.25, wider face-classification heads (HEAD_GAIN) with the
    logit offsets of SYNTH_LOGIT_SHIFT, and narrower regression heads (x0.3), so that on smooth synthetic
    images the face probabilities spread across every stage's threshold (each stage keeps some candidates
    and drops others) and boxes stay near their cell.  calibrated=True also lowers the face logits by
    CALIBRATED_LOGIT_SHIFT (trained-detector box volumes, tools/calibrate_mtcnn.py)."""
    from .weights import splitmix_uniform
    out = {}
    for net, specs in MTCNN_SPECS.items():
        for name, shape in specs:
            key = f"{net}.{name}"
            u = splitmix_uniform(seed, key, int(np.prod(shape))).reshape(shape)
            if name.startswith("prelu"):
                v = np.full(shape, 0.25)
            else:
                wshape = dict(specs)[name.replace(".bias", ".weight")]
                fan_in = int(np.prod(wshape[1:]))
                v = (2 * u - 1) / np.sqrt(fan_in)
                head = name.split(".")[0]
                if head in HEAD_GAIN:
                    v = v * HEAD_GAIN[head]
                elif head in ("conv4_2", "dense5_2", "dense6_2", "dense6_3"):
                    v = v * 0.3
            if key in SYNTH_LOGIT_SHIFT:  # (background, face) logit offsets of the synthetic heads
                v = v + np.asarray(SYNTH_LOGIT_SHIFT[key])
            if calibrated and key in CALIBRATED_LOGIT_SHIFT:
                d = CALIBRATED_LOGIT_SHIFT[key]
                v = v + np.asarray([d / 2, -d / 2])
            out[key] = v.astype(np.float32)
    return out


def load_mtcnn_state(directory: str) -> Dict[str, np.ndarray]:
    """facenet-pytorch's data/pnet.pt, rnet.pt, onet.pt (state dicts) -> {"pnet.<param>": array, ...}."""
    import torch
    out = {}
    for net in MTCNN_SPECS:
        sd = torch.load(os.path.join(directory, f"{net}.pt"), map_location="cpu", weights_only=True)
        for name, shape in MTCNN_SPECS[net]:
            v = np.asarray(sd[name].float().numpy(), np.float32)
            if v.shape != shape:
                raise ValueError(f"{net}.{name}: shape {v.shape}, expected {shape}")
            out[f"{net}.{name}"] = v
    return out


def pool_ceil_out(n: int, k: int, s: int) -> int:
    """MaxPool2d(k, s, ceil_mode=True) output size (mtcnn.hip pool_ceil_out)."""
    o = -(-(n - k) // s) + 1
    if (o - 1) * s >= n:
        o -= 1
    return max(o, 1)


def pyramid_scales(h: int, w: int, minsize: int = MIN_FACE, factor: float = FACTOR) -> List[float]:
    """detect_face's scale pyramid: 12 / minsize, times factor while the short side stays >= 12."""
    m = 12.0 / minsize
    minl = min(h, w) * m
    scales, s = [], m
    while minl >= 12:
        scales.append(s)
        s *= factor
        minl *= factor
    return scales


# ------------------------------------------------------------------------------ host box logic
# Optional per-stage timing of detect_face (tools/mtcnn_bench.py): a dict here receives ms and counts
STATS = None


def _acc(key, t0, n=None):
    if STATS is not None:
        STATS[key] = STATS.get(key, 0.0) + (time.perf_counter() - t0) * 1e3
        if n is not None:
            STATS[key + "_n"] = STATS.get(key + "_n", 0) + int(n)


def _cnt(key, n):
    if STATS is not None:
        STATS[key] = STATS.get(key, 0) + int(n)


def nms(boxes: np.ndarray, scores: np.ndarray, thresh: float, mode: str = "iou") -> np.ndarray:
    """Greedy non-maximum suppression.  mode "iou": torchvision.ops.nms (score descending, equal scores
    in index order, areas (x2 - x1)(y2 - y1), suppress IoU > thresh: a 0 / 0 IoU keeps the box); mode "min":
    detect_face.nms_numpy's 'Min' (+1-pixel areas, np.argsort order from the highest score, keep overlap /
    min-area <= thresh: a NaN drops the box).  The score order is numpy's; the greedy pass is libfrhip's grid-bucketed fr_nms_host (the same
    float32 overlap arithmetic, O(n) instead of O(kept x n): PNet proposes ~10^5 windows per 1080p level)."""
    import ctypes
    from . import _native as N
    n = len(boxes)
    if n == 0:
        return np.zeros((0,), np.int64)
    t0 = time.perf_counter()
    order = np.argsort(-scores, kind="stable") if mode == "iou" else np.argsort(scores)[::-1]
    b = np.ascontiguousarray(boxes[:, :4], dtype=np.float32)
    order = np.ascontiguousarray(order, dtype=np.int64)
    keep = np.empty(n, np.int64)
    nk = ctypes.c_int64(0)
    N.check(N.lib().fr_nms_host(b.ctypes.data, n, order.ctypes.data, float(thresh), int(mode == "min"),
                                keep.ctypes.data, ctypes.byref(nk)), "fr_nms_host")
    _acc("nms_ms", t0, n)
    return keep[: nk.value].copy()


def batched_nms(boxes: np.ndarray, scores: np.ndarray, image_inds: np.ndarray, thresh: float,
                mode: str = "iou") -> np.ndarray:
    """NMS per image, through the coordinate-offset trick of torchvision's batched_nms / detect_face's
    batched_nms_numpy (boxes of different images never overlap)."""
    if len(boxes) == 0:
        return np.zeros((0,), np.int64)
    off = image_inds.astype(np.float32) * (boxes[:, :4].max() + np.float32(1))
    return nms((boxes[:, :4] + off[:, None]).astype(np.float32), scores, thresh, mode)


def _bbreg(b: np.ndarray, reg: np.ndarray) -> np.ndarray:
    w = b[:, 2] - b[:, 0] + np.float32(1)
    h = b[:, 3] - b[:, 1] + np.float32(1)
    b = b.copy()
    b[:, 0], b[:, 1] = b[:, 0] + reg[:, 0] * w, b[:, 1] + reg[:, 1] * h
    b[:, 2], b[:, 3] = b[:, 2] + reg[:, 2] * w, b[:, 3] + reg[:, 3] * h
    return b


def _rerec(b: np.ndarray) -> np.ndarray:
    b = b.copy()
    h = b[:, 3] - b[:, 1]
    w = b[:, 2] - b[:, 0]
    l = np.maximum(w, h)
    b[:, 0] = b[:, 0] + w * np.float32(0.5) - l * np.float32(0.5)
    b[:, 1] = b[:, 1] + h * np.float32(0.5) - l * np.float32(0.5)
    b[:, 2] = b[:, 0] + l
    b[:, 3] = b[:, 1] + l
    return b


def _pad(b: np.ndarray, w: int, h: int):
    t = np.trunc(b[:, :4]).astype(np.int32)
    x, y, ex, ey = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
    x[x < 1] = 1
    y[y < 1] = 1
    ex[ex > w] = w
    ey[ey > h] = h
    return y, ey, x, ex


def detect_face(imgs, resample, pnet, rnet, onet, minsize: int = MIN_FACE, thresholds=THRESHOLDS,
                factor: float = FACTOR):
    """facenet-pytorch's detect_face (models/utils/detect_face.py, 2.5.x) around four callables:
    resample(imgs, regions [n, 5] (image, y0, x0, h, w), oh, ow) -> normalised NHWC crops, and the three
    nets (NHWC in; pnet -> [B, h, w, 6], rnet -> [n, 6], onet -> [n, 16]: face-softmax pair, box
    regression, landmarks), each returning a tensor with .cpu().  imgs: RGB u8 [B, H, W, 3].  Returns per
    image boxes [n, 5] (x1, y1, x2, y2, prob) and landmarks [n, 5, 2]; all box arithmetic in float32."""
    B, h, w, _ = imgs.shape
    th = thresholds
    f32 = np.float32
    boxes, inds, picks, offset = [], [], [], 0
    for scale in pyramid_scales(h, w, minsize, factor):
        hs, ws = int(h * scale + 1), int(w * scale + 1)
        t0 = time.perf_counter()
        x = resample(imgs, np.array([[b, 0, 0, h, w] for b in range(B)]), hs, ws)
        out = pnet(x).cpu().numpy()  # [B, hh, ww, 6]
        _acc("pnet_ms", t0, out.shape[0] * out.shape[1] * out.shape[2])
        prob = out[..., 1]
        bi, yy, xx = np.nonzero(prob >= f32(th[0]))
        sc = f32(scale)
        cell = np.stack([xx, yy], 1).astype(f32)
        q1 = np.floor((f32(2) * cell + f32(1)) / sc)
        q2 = np.floor((f32(2) * cell + f32(12)) / sc)
        bs = np.concatenate([q1, q2, prob[bi, yy, xx][:, None], out[bi, yy, xx, 2:6]], 1).astype(f32)
        _cnt("pnet_pass_n", len(bs))
        boxes.append(bs)
        inds.append(bi)
        picks.append(batched_nms(bs, bs[:, 4], bi, 0.5) + offset)
        offset += len(bs)
    boxes = np.concatenate(boxes, 0) if boxes else np.zeros((0, 9), f32)
    inds = np.concatenate(inds, 0) if inds else np.zeros((0,), np.int64)
    pk = np.concatenate(picks, 0) if picks else np.zeros((0,), np.int64)
    boxes, inds = boxes[pk], inds[pk]
    pk = batched_nms(boxes, boxes[:, 4], inds, 0.7)
    boxes, inds = boxes[pk], inds[pk]
    regw, regh = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
    boxes = np.stack([boxes[:, 0] + boxes[:, 5] * regw, boxes[:, 1] + boxes[:, 6] * regh,
                      boxes[:, 2] + boxes[:, 7] * regw, boxes[:, 3] + boxes[:, 8] * regh, boxes[:, 4]], 1).astype(f32)
    boxes = _rerec(boxes)
    points = np.zeros((0, 5, 2), f32)

    def crops(bx, size):
        y, ey, x, ex = _pad(bx, w, h)
        ok = (ey > y - 1) & (ex > x - 1)
        reg = np.stack([inds, y - 1, x - 1, ey - y + 1, ex - x + 1], 1)[ok]
        return resample(imgs, reg, size, size), ok

    if len(boxes):
        t0 = time.perf_counter()
        x, ok = crops(boxes, 24)
        boxes, inds = boxes[ok], inds[ok]
        out = rnet(x).cpu().numpy()
        _acc("rnet_ms", t0, len(out))
        score = out[:, 1]
        ip = score > f32(th[1])
        boxes = np.concatenate([boxes[ip, :4], score[ip, None]], 1)
        inds, mv = inds[ip], out[ip, 2:6]
        pk = batched_nms(boxes, boxes[:, 4], inds, 0.7)
        boxes, inds, mv = boxes[pk], inds[pk], mv[pk]
        boxes = _rerec(_bbreg(boxes, mv))
    if len(boxes):
        t0 = time.perf_counter()
        x, ok = crops(boxes, 48)
        boxes, inds = boxes[ok], inds[ok]
        out = onet(x).cpu().numpy()
        _acc("onet_ms", t0, len(out))
        score = out[:, 1]
        ip = score > f32(th[2])
        boxes = np.concatenate([boxes[ip, :4], score[ip, None]], 1)
        inds, mv, pts = inds[ip], out[ip, 2:6], out[ip, 6:16]
        w_i = boxes[:, 2] - boxes[:, 0] + f32(1)
        h_i = boxes[:, 3] - boxes[:, 1] + f32(1)
        px = w_i[:, None] * pts[:, :5] + boxes[:, 0:1] - f32(1)
        py = h_i[:, None] * pts[:, 5:10] + boxes[:, 1:2] - f32(1)
        points = np.stack([px, py], 2).astype(f32)
        boxes = _bbreg(boxes, mv)
        pk = batched_nms(boxes, boxes[:, 4], inds, 0.7, "min")
        boxes, inds, points = boxes[pk], inds[pk], points[pk]
    _cnt("final_n", len(boxes))
    return [boxes[inds == b] for b in range(B)], [points[inds == b] for b in range(B)]


# ------------------------------------------------------------------------------ device nets
class DeviceMTCNN:
    """facenet-pytorch's MTCNN.detect on the device: the P/R/O-nets of ``state`` (synth_mtcnn_state /
    load_mtcnn_state layout) as f32 NHWC launches of mtcnn.hip."""

    def __init__(self, state: Dict[str, np.ndarray], device: int = 0, min_face_size: int = MIN_FACE,
                 thresholds: Sequence[float] = THRESHOLDS, factor: float = FACTOR, select_largest: bool = True):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("DeviceMTCNN needs a ROCm GPU; there is deliberately no CPU fallback")
        self.device = torch.device("cuda", device)
        self.min_face_size, self.thresholds, self.factor = min_face_size, tuple(thresholds), factor
        self.select_largest = select_largest
        dev = self.device

        def t(a):
            return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32)).to(dev)

        def conv(net, name):  # [Cout, Cin, kh, kw] -> [Cout, kh, kw, Cin]
            w = state[f"{net}.{name}.weight"]
            return t(w.transpose(0, 2, 3, 1)), t(state[f"{net}.{name}.bias"]), w.shape

        def dense_nhwc(net, name, H, W, C):  # columns from the (w, h, c) flatten of permute(0, 3, 2, 1) to NHWC
            w = state[f"{net}.{name}.weight"]
            idx = np.arange(H * W * C).reshape(W, H, C).transpose(1, 0, 2).reshape(-1)
            return t(w[:, idx]), t(state[f"{net}.{name}.bias"])

        def head(net, names, C):
            w = np.concatenate([state[f"{net}.{n}.weight"].reshape(-1, C) for n in names], 0)
            b = np.concatenate([state[f"{net}.{n}.bias"] for n in names], 0)
            return t(w), t(b)

        pr = lambda net, i: t(state[f"{net}.prelu{i}.weight"])  # noqa: E731
        self.p = {"c": [conv("pnet", f"conv{i}") for i in (1, 2, 3)], "a": [pr("pnet", i) for i in (1, 2, 3)],
                  "h": head("pnet", ("conv4_1", "conv4_2"), 32)}
        self.r = {"c": [conv("rnet", f"conv{i}") for i in (1, 2, 3)], "a": [pr("rnet", i) for i in (1, 2, 3, 4)],
                  "d": dense_nhwc("rnet", "dense4", 3, 3, 64), "h": head("rnet", ("dense5_1", "dense5_2"), 128)}
        self.o = {"c": [conv("onet", f"conv{i}") for i in (1, 2, 3, 4)], "a": [pr("onet", i) for i in (1, 2, 3, 4, 5)],
                  "d": dense_nhwc("onet", "dense5", 3, 3, 128),
                  "h": head("onet", ("dense6_1", "dense6_2", "dense6_3"), 256)}

    # -- launches --------------------------------------------------------------------------------
    def _s(self):
        return N.stream_ptr(self.device)

    def _conv(self, x, layer, slope):
        import torch
        w, b, shape = layer
        B, H, W, C = x.shape
        cout, _, kh, kw = shape
        y = torch.empty((B, H - kh + 1, W - kw + 1, cout), dtype=torch.float32, device=self.device)
        N.check(N.lib().fr_mtcnn_conv(N.ptr(x), B, H, W, C, N.ptr(w), N.ptr(b), N.ptr(slope), cout, kh, kw, N.ptr(y),
                                      self._s()), "fr_mtcnn_conv")
        return y

    def _pool(self, x, k, s):
        import torch
        B, H, W, C = x.shape
        y = torch.empty((B, pool_ceil_out(H, k, s), pool_ceil_out(W, k, s), C), dtype=torch.float32, device=self.device)
        N.check(N.lib().fr_mtcnn_maxpool(N.ptr(x), B, H, W, C, k, s, N.ptr(y), self._s()), "fr_mtcnn_maxpool")
        return y

    def _dense(self, x, layer, slope):
        import torch
        w, b = layer
        B, K = x.shape[0], int(np.prod(x.shape[1:]))
        y = torch.empty((B, w.shape[0]), dtype=torch.float32, device=self.device)
        N.check(N.lib().fr_mtcnn_dense(N.ptr(x), B, K, N.ptr(w), N.ptr(b), N.ptr(slope), int(w.shape[0]), N.ptr(y),
                                       self._s()), "fr_mtcnn_dense")
        return y

    def _head(self, x, layer):
        import torch
        w, b = layer
        M, C = int(np.prod(x.shape[:-1])), int(x.shape[-1])
        y = torch.empty(tuple(x.shape[:-1]) + (int(w.shape[0]),), dtype=torch.float32, device=self.device)
        N.check(N.lib().fr_mtcnn_head(N.ptr(x), M, C, N.ptr(w), N.ptr(b), int(w.shape[0]), N.ptr(y), self._s()),
                "fr_mtcnn_head")
        return y

    def resample(self, imgs_dev, regions: np.ndarray, oh: int, ow: int):
        """Area-resampled, normalised f32 NHWC crops of u8 images (regions [n, 5]: image, y0, x0, h, w)."""
        import torch
        _, H, W, _ = imgs_dev.shape
        reg = torch.as_tensor(np.ascontiguousarray(regions, dtype=np.int32)).to(self.device)
        out = torch.empty((len(regions), oh, ow, 3), dtype=torch.float32, device=self.device)
        N.check(N.lib().fr_area_resample_u8(N.ptr(imgs_dev), H, W, N.ptr(reg), len(regions), oh, ow, N.ptr(out),
                                            self._s()), "fr_area_resample_u8")
        return out

    def pnet(self, x):
        p = self.p
        x = self._pool(self._conv(x, p["c"][0], p["a"][0]), 2, 2)
        x = self._conv(self._conv(x, p["c"][1], p["a"][1]), p["c"][2], p["a"][2])
        return self._head(x, p["h"])  # [B, h, w, 6]: prob(bg), prob(face), reg x4

    def rnet(self, x):
        r = self.r
        x = self._pool(self._conv(x, r["c"][0], r["a"][0]), 3, 2)
        x = self._pool(self._conv(x, r["c"][1], r["a"][1]), 3, 2)
        x = self._conv(x, r["c"][2], r["a"][2])
        return self._head(self._dense(x, r["d"], r["a"][3]), r["h"])  # [n, 6]

    def onet(self, x):
        o = self.o
        x = self._pool(self._conv(x, o["c"][0], o["a"][0]), 3, 2)
        x = self._pool(self._conv(x, o["c"][1], o["a"][1]), 3, 2)
        x = self._pool(self._conv(x, o["c"][2], o["a"][2]), 2, 2)
        x = self._conv(x, o["c"][3], o["a"][3])
        return self._head(self._dense(x, o["d"], o["a"][4]), o["h"])  # [n, 16]: probs, reg x4, landmarks x10

    # -- detect_face -----------------------------------------------------------------------------
    def detect_face(self, imgs_u8):
        """detect_face (facenet-pytorch 2.5.x) on equal-size RGB u8 images [B, H, W, 3] (numpy or device):
        per image, boxes [n, 5] (x1, y1, x2, y2, prob) and landmarks [n, 5, 2]."""
        import torch
        imgs = torch.as_tensor(imgs_u8) if not torch.is_tensor(imgs_u8) else imgs_u8
        imgs = imgs.to(self.device).contiguous()
        return detect_face(imgs, self.resample, self.pnet, self.rnet, self.onet, self.min_face_size,
                           self.thresholds, self.factor)

    def detect(self, img_rgb_u8, landmarks: bool = True):
        """MTCNN.detect(img, landmarks=True) for one RGB u8 image [H, W, 3]: (boxes [n, 4] or None, probs,
        points [n, 5, 2]), the largest box first when select_largest."""
        boxes, points = self.detect_face(np.asarray(img_rgb_u8)[None])
        box, point = boxes[0], points[0]
        if len(box) == 0:
            return (None, [None], None) if landmarks else (None, [None])
        if self.select_largest:
            order = np.argsort((box[:, 2] - box[:, 0]) * (box[:, 3] - box[:, 1]))[::-1]
            box, point = box[order], point[order]
        return (box[:, :4], box[:, 4], point) if landmarks else (box[:, :4], box[:, 4])


class FaceDetector:
    """The reference's ``FaceDetector`` (preprocessing/face_detector.py:21-116) with the MTCNN backend on the
    device.  ``detect(image_bgr)`` -> {'bbox', 'confidence', 'landmarks'} or None; ``crop_face``."""

    DEFAULT_CONFIDENCE_THRESHOLD = 0.9
    MIN_FACE_SIZE = 20

    def __init__(self, backend: str = "mtcnn", device: str = "cuda", confidence_threshold: float = 0.9,
                 min_face_size: int = 20, select_largest: bool = True, mtcnn_state: Optional[Dict] = None,
                 weights_dir: Optional[str] = None):
        from .extract_embeddings import _device_index
        self.backend = backend.lower()
        if self.backend != "mtcnn":
            raise ValueError(f"Backend khong ho tro: {self.backend} (the device detector is MTCNN)")
        self.device = device
        self.confidence_threshold = confidence_threshold
        self.min_face_size = min_face_size
        self.select_largest = select_largest
        if mtcnn_state is None:
            weights_dir = weights_dir or os.environ.get("FR_MTCNN_WEIGHTS")
            if not weights_dir:
                raise ImportError("MTCNN weights (facenet-pytorch's pnet.pt / rnet.pt / onet.pt) not available: pass "
                                  "weights_dir= or set FR_MTCNN_WEIGHTS")
            mtcnn_state = load_mtcnn_state(weights_dir)
        self.detector = DeviceMTCNN(mtcnn_state, device=_device_index(device), min_face_size=min_face_size)
        print(f"[OK] MTCNN initialized on {device} (device P/R/O-nets)")

    def detect(self, image: np.ndarray) -> Optional[Dict]:
        """_detect_mtcnn: BGR u8 [H, W, 3] -> the chosen face or None (face_detector.py:144-210)."""
        if image is None or image.size == 0:
            return None
        rgb = np.ascontiguousarray(image[..., ::-1]) if image.ndim == 3 and image.shape[2] == 3 else image
        return self.detect_rgb(rgb)

    def detect_rgb(self, rgb: np.ndarray) -> Optional[Dict]:
        boxes, probs, landmarks = self.detector.detect(rgb, landmarks=True)
        if boxes is None or len(boxes) == 0:
            return None
        probs = np.asarray(probs)
        valid = probs >= self.confidence_threshold
        if not np.any(valid):
            return None
        boxes, probs, landmarks = boxes[valid], probs[valid], landmarks[valid]
        faces = [i for i, b in enumerate(boxes) if min(b[2] - b[0], b[3] - b[1]) >= self.min_face_size]
        if not faces:
            return None
        if self.select_largest and len(faces) > 1:
            best = faces[int(np.argmax([(boxes[i][2] - boxes[i][0]) * (boxes[i][3] - boxes[i][1]) for i in faces]))]
        else:
            best = faces[0]
        b, lm = boxes[best], landmarks[best]
        return {"bbox": [int(b[0]), int(b[1]), int(b[2]), int(b[3])], "confidence": float(probs[best]),
                "landmarks": {n: (float(lm[k][0]), float(lm[k][1])) for k, n in enumerate(LANDMARK_NAMES)}}

    def crop_face(self, image: np.ndarray, margin: float = 0.3, target_size: Optional[Tuple[int, int]] = None):
        """Detect, crop with a margin (face_detector.py:367-407).  The resize to target_size uses the device
        PIL-exact bilinear resize (align.resize_u8), not cv2.resize's INTER_LINEAR (cv2 is absent: this
        fallback's pixels are not pinned to the reference)."""
        det = self.detect(image)
        if det is None:
            return None
        x1, y1, x2, y2 = det["bbox"]
        h, w = image.shape[:2]
        mw, mh = int((x2 - x1) * margin), int((y2 - y1) * margin)
        x1, y1, x2, y2 = max(0, x1 - mw), max(0, y1 - mh), min(w, x2 + mw), min(h, y2 + mh)
        cropped = image[y1:y2, x1:x2]
        if target_size and cropped.size:
            import torch
            from .align import resize_u8
            t = torch.as_tensor(np.ascontiguousarray(cropped))[None].to(self.detector.device)
            cropped = resize_u8(t, target_size[1], target_size[0])[0].cpu().numpy()
        return cropped
