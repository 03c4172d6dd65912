"""CPU restatements of the crop-preparation steps (TEST INFRASTRUCTURE ONLY).

* pillow_resize: PIL Image.resize(size, BILINEAR) for RGB u8 (Pillow libImaging/Resample.c,
  ImagingResampleInner / precompute_coeffs / normalize_coeffs_8bpc / ImagingResample{Horizontal,Vertical}
  _8bpc), used by the reference's get_transform Resize (inference/extract_embeddings.py:170-185).  PIL is
  installed, so tests/test_preprocess.py pins this restatement to PIL itself.
* cv2_warp_affine: cv2.warpAffine(img, M, (OW, OH), borderValue=0), INTER_LINEAR / BORDER_CONSTANT,
  restating OpenCV's fixed-point path (imgproc/src/imgwarp.cpp: warpAffine's matrix inversion,
  WarpAffineInvoker with AB_BITS = 10 / INTER_BITS = 5, cvRound, initInterTab2D(INTER_LINEAR, fixpt),
  remapBilinear with FixedPtCast<int, uchar, 15>), used by align_face (extract_embeddings.py:216-242,
  recognition_engine.py:169-204).  cv2 is not installed and the reference holds no warped fixtures, so
  this one is parity unpinned.
Pure numpy, vectorised; sizes up to a few hundred pixels run in milliseconds."""
from __future__ import annotations

import math

import numpy as np

PB = 22


def _coeffs(in_size: int, out_size: int):
    in0, in1 = 0.0, float(np.float32(in_size))
    scale = (in1 - in0) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)  # C (int) cast: truncation toward zero
        xmin = max(xmin, 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = []
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w = 1.0 - t if t < 1.0 else 0.0
            k.append(w)
            ww += w
        if ww != 0.0:
            k = [v / ww for v in k]
        for x, v in enumerate(k):
            kk[xx, x] = int(-0.5 + v * (1 << PB)) if v < 0 else int(0.5 + v * (1 << PB))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(v: np.ndarray) -> np.ndarray:
    return np.clip(v >> PB, 0, 255).astype(np.uint8)


def pillow_resize(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """img: u8 [H, W, 3] -> u8 [out_h, out_w, 3]."""
    H, W = img.shape[:2]
    bh, kh = _coeffs(W, out_w)
    bv, kv = _coeffs(H, out_h)
    need_h, need_v = out_w != W, out_h != H
    src = img.astype(np.int64)
    if need_h:
        y0 = bv[0, 0]
        y1 = bv[-1, 0] + bv[-1, 1]
        bv = bv.copy()
        bv[:, 0] -= y0
        rows = src[y0:y1]
        tmp = np.empty((y1 - y0, out_w, 3), np.int64)
        for x in range(out_w):
            xmin, n = bh[x]
            acc = (1 << (PB - 1)) + np.einsum("rtc,t->rc", rows[:, xmin:xmin + n], kh[x, :n])
            tmp[:, x] = _clip8(acc)
        src = tmp
    if need_v:
        out = np.empty((out_h, src.shape[1], 3), np.uint8)
        for y in range(out_h):
            ymin, n = bv[y]
            acc = (1 << (PB - 1)) + np.einsum("tkc,t->kc", src[ymin:ymin + n], kv[y, :n])
            out[y] = _clip8(acc)
        return out
    return src.astype(np.uint8)


def cv2_warp_affine(img: np.ndarray, M: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """img: u8 [H, W, C]; M: forward 2x3 (float64)."""
    H, W, C = img.shape
    m = [float(v) for v in np.asarray(M, np.float64).reshape(6)]
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = m[4] * D, m[0] * D
    m[0] = A11
    m[1] *= -D
    m[3] *= -D
    m[4] = A22
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    AB = 1024
    rd = AB // 32 // 2
    y = np.arange(out_h, dtype=np.float64)[:, None]
    x = np.arange(out_w, dtype=np.float64)[None, :]
    rint = lambda v: np.rint(v).astype(np.int64)  # cvRound: round half to even
    X0 = rint((m[1] * y + m[2]) * AB) + rd
    Y0 = rint((m[4] * y + m[5]) * AB) + rd
    X = (X0 + rint(m[0] * x * AB)) >> 5
    Y = (Y0 + rint(m[3] * x * AB)) >> 5
    sx, sy, tx, ty = X >> 5, Y >> 5, X & 31, Y & 31
    w = [(32 - ty) * (32 - tx) * 32, (32 - ty) * tx * 32, ty * (32 - tx) * 32, ty * tx * 32]
    src = img.astype(np.int64)

    def px(xx, yy):
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        v = src[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)]
        return np.where(ok[..., None], v, 0)

    acc = (px(sx, sy) * w[0][..., None] + px(sx + 1, sy) * w[1][..., None] +
           px(sx, sy + 1) * w[2][..., None] + px(sx + 1, sy + 1) * w[3][..., None])
    out = np.clip((acc + (1 << 14)) >> 15, 0, 255).astype(np.uint8)
    outside = (sx >= W) | (sx + 1 < 0) | (sy >= H) | (sy + 1 < 0)
    out[outside] = 0
    return out
