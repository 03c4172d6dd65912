"""Deterministic synthetic aligned-crop batches (no datasets are reachable offline).

``synthetic_crops(n, size, seed)`` returns u8 [n, size, size, 3] RGB crops: a random low-resolution
colour field (6x6 control points, bilinear upsampled) plus uniform pixel noise.  Unlike i.i.d.
uniform noise, two such crops differ in their global statistics, so backbones that end in a global
average pool (ResNet-50 ArcFace, InceptionResnetV1) produce well-separated embeddings instead of the
near-identical pooled features of i.i.d. noise (DESIGN.md §5 'Synthetic inputs').
Pure numpy, so every machine regenerates the same bytes.
"""
from __future__ import annotations

import numpy as np


def _lin_weights(n_out: int, n_in: int):
    # align_corners=False bilinear sampling positions
    x = (np.arange(n_out) + 0.5) * (n_in / n_out) - 0.5
    x = np.clip(x, 0, n_in - 1)
    i0 = np.floor(x).astype(np.int64)
    i1 = np.minimum(i0 + 1, n_in - 1)
    w1 = (x - i0).astype(np.float32)
    return i0, i1, w1


def synthetic_crops(n: int, size: int = 112, seed: int = 0, grid: int = 6, noise: float = 24.0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    low = rng.uniform(0, 255, (n, grid, grid, 3)).astype(np.float32)
    i0, i1, w1 = _lin_weights(size, grid)
    rows = low[:, i0] * (1 - w1)[None, :, None, None] + low[:, i1] * w1[None, :, None, None]
    img = rows[:, :, i0] * (1 - w1)[None, None, :, None] + rows[:, :, i1] * w1[None, None, :, None]
    img = img + rng.uniform(-noise, noise, img.shape).astype(np.float32)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


GALLERY_BLOCK = 1 << 16  # rows per independently seeded block of synthetic_gallery_rows


def synthetic_gallery_rows(lo: int, hi: int, device, dim: int = 512, seed: int = 1):
    """Rows [lo, hi) of the synthetic random unit-norm gallery (standard-normal rows,
    L2-normalized), generated on the device in GALLERY_BLOCK-row blocks, each seeded by (seed, block).
    Any shard of a 1M x 512 gallery is reproduced on its own rank without materialising the whole
    2 GB matrix anywhere, and the rows do not depend on how the gallery is sharded."""
    import torch

    out = torch.empty((hi - lo, dim), dtype=torch.float32, device=device)
    for b in range(lo // GALLERY_BLOCK, (hi + GALLERY_BLOCK - 1) // GALLERY_BLOCK):
        g = torch.Generator(device=device)
        g.manual_seed(seed * 1_000_003 + b)
        blk = torch.randn((GALLERY_BLOCK, dim), generator=g, device=device)
        s, e = max(lo, b * GALLERY_BLOCK), min(hi, (b + 1) * GALLERY_BLOCK)
        out[s - lo:e - lo] = blk[s - b * GALLERY_BLOCK:e - b * GALLERY_BLOCK]
    out /= out.norm(dim=1, keepdim=True)
    return out


def planted_gallery(probe_emb: np.ndarray, n_rows: int, seed: int = 1, jitter: float = 0.05) -> np.ndarray:
    """Unit-norm gallery [n_rows, D]: row j < len(probe_emb) = normalize(e_j + jitter*noise)
    (a planted match for probe j), the rest random directions."""
    rng = np.random.default_rng(seed)
    d = probe_emb.shape[1]
    G = rng.standard_normal((n_rows, d)).astype(np.float32)
    k = min(len(probe_emb), n_rows)
    G[:k] = probe_emb[:k] + jitter * rng.standard_normal((k, d)).astype(np.float32)
    G /= np.linalg.norm(G, axis=1, keepdims=True)
    return G
