"""Face alignment and resizing on the device: the steps between a decoded image and
the aligned crop the embedding path takes.

Reference → here:
  align_face (inference/extract_embeddings.py:216-242, recognition_engine.py:169-204):
      SimilarityTransform().estimate(src, ARCFACE_TEMPLATE)   -> similarity_transform() (host, 5 points)
      cv2.warpAffine(image, M, (112, 112), borderValue=0)     -> fr_warp_affine_u8 (device, batched)
  get_transform / get_facenet_transform Resize (extract_embeddings.py:170-185):
      PIL Image.resize((S, S), Image.BILINEAR)                -> fr_resize_u8 (device, batched, PIL-exact)
The landmark detector (MTCNN) stays out of scope: landmarks come from the caller, as the reference's
align_face receives them."""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np

from . import _native as N

ARCFACE_TEMPLATE = np.array([[38.2946, 51.6963], [73.5318, 51.5014], [56.0252, 71.7366],
                             [41.5493, 92.3655], [70.7299, 92.2041]], dtype=np.float32)
LANDMARK_KEYS = ("left_eye", "right_eye", "nose", "left_mouth", "right_mouth")


def similarity_transform(src: np.ndarray, dst: np.ndarray = ARCFACE_TEMPLATE) -> np.ndarray:
    """skimage.transform.SimilarityTransform().estimate(src, dst).params (3x3, float64): the closed-form
    least-squares similarity of Umeyama (1991), as skimage's _umeyama(src, dst, estimate_scale=True)
    computes it (scikit-image is not installed: restated, parity unpinned)."""
    src = np.asarray(src, dtype=np.float64)
    dst = np.asarray(dst, dtype=np.float64)
    num, dim = src.shape
    src_mean, dst_mean = src.mean(axis=0), dst.mean(axis=0)
    src_d, dst_d = src - src_mean, dst - dst_mean
    A = dst_d.T @ src_d / num
    d = np.ones((dim,), dtype=np.float64)
    if np.linalg.det(A) < 0:
        d[dim - 1] = -1
    T = np.eye(dim + 1, dtype=np.float64)
    U, S, V = np.linalg.svd(A)
    rank = np.linalg.matrix_rank(A)
    if rank == 0:
        return np.nan * T
    if rank == dim - 1:
        if np.linalg.det(U) * np.linalg.det(V) > 0:
            T[:dim, :dim] = U @ V
        else:
            s = d[dim - 1]
            d[dim - 1] = -1
            T[:dim, :dim] = U @ np.diag(d) @ V
            d[dim - 1] = s
    else:
        T[:dim, :dim] = U @ np.diag(d) @ V
    scale = 1.0 / src_d.var(axis=0).sum() * (S @ d)
    T[:dim, dim] = dst_mean - scale * (T[:dim, :dim] @ src_mean.T)
    T[:dim, :dim] *= scale
    return T


def landmarks_to_src(landmarks: Dict) -> np.ndarray:
    """The reference's src array from a landmark dict (missing points -> [0, 0])."""
    return np.array([landmarks.get(k, [0, 0]) for k in LANDMARK_KEYS], dtype=np.float32)


def resize_u8(images, out_h: int, out_w: int):
    """Device PIL-exact bilinear resize: images cuda u8 [B, H, W, 3] -> cuda u8 [B, out_h, out_w, 3]."""
    import torch
    x = images.contiguous()
    B, H, W, _ = x.shape
    out = torch.empty((B, out_h, out_w, 3), dtype=torch.uint8, device=x.device)
    nws = int(N.lib().fr_resize_u8_workspace(B, H, W, out_h, out_w))
    ws = torch.empty((max(nws, 1),), dtype=torch.uint8, device=x.device)
    N.check(N.lib().fr_resize_u8(N.ptr(x), B, H, W, N.ptr(out), out_h, out_w, N.ptr(ws), nws, N.stream_ptr(x.device)),
            "fr_resize_u8")
    return out


def warp_affine_u8(images, matrices, out_h: int = 112, out_w: int = 112):
    """Device cv2.warpAffine(..., borderValue=0): images cuda u8 [B, H, W, 3], matrices [B, 2, 3] forward
    (host or device, float64) -> cuda u8 [B, out_h, out_w, 3]."""
    import torch
    x = images.contiguous()
    B, H, W, _ = x.shape
    M = torch.as_tensor(np.asarray(matrices, dtype=np.float64).reshape(B, 6) if not torch.is_tensor(matrices)
                        else matrices.double().reshape(B, 6)).to(x.device).contiguous()
    out = torch.empty((B, out_h, out_w, 3), dtype=torch.uint8, device=x.device)
    N.check(N.lib().fr_warp_affine_u8(N.ptr(x), B, H, W, N.ptr(M), N.ptr(out), out_h, out_w, N.stream_ptr(x.device)),
            "fr_warp_affine_u8")
    return out


def align_faces(images, landmarks: Sequence[Dict], out_size: int = 112):
    """align_face for a batch of same-size images (cuda u8 [B, H, W, 3]) with one landmark dict each:
    similarity to ARCFACE_TEMPLATE on the host, one warp launch for the batch.  Returns (crops cuda u8
    [B, 112, 112, 3], ok [B] bool); a face whose landmarks are all zero is not aligned (the reference
    returns None for it) and its crop is left zero."""
    mats, ok = [], []
    for lm in landmarks:
        src = landmarks_to_src(lm)
        good = not np.all(src == 0)
        T = similarity_transform(src) if good else np.eye(3)
        good = good and np.all(np.isfinite(T))
        mats.append(T[:2] if good else np.array([[1.0, 0, 1e5], [0, 1.0, 1e5]]))  # samples far outside: zeros
        ok.append(good)
    return warp_affine_u8(images, np.stack(mats), out_size, out_size), np.array(ok)
