"""Device-resident gallery with exact inner-product top-k (libfrhip match kernel).

Drop-in for the reference's three match paths:
  * ``RecognitionEngine.recognize_with_db`` — per-row ``cosine_similarity`` loop + stable
    ``sort(reverse=True)`` (inference/recognition_engine.py:267-289, :41-63);
  * FAISS ``IndexFlatIP`` (``build_faiss_index`` extract_embeddings.py:595-645, searched in
    recognition_engine.py:291-326) — ``DeviceGallery`` exposes the same ``add``/``search``/
    ``ntotal`` surface, ``search`` returning (scores, ids) with ids int64 and -1 padding;
  * the notebook's batched ``np.dot(emb, P.T)`` + ``argmax``/``argsort[:, -5:]``.
Order is (score desc, index asc) everywhere, i.e. ``np.argmax``'s first-max rule and the
stable sort's insertion order on ties.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _native as N


class DeviceGallery:
    def __init__(self, rows=None, dim: int = 512, device: int = 0, index_base: int = 0, handle=None,
                 x3_min_rows: Optional[int] = None):
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("DeviceGallery needs a ROCm GPU; there is deliberately no CPU fallback")
        self.device = torch.device("cuda", device)
        self.d = dim
        self.index_base = int(index_base)
        self._own = handle is None
        if handle is None:
            h = ctypes.c_void_p()
            N.check(N.lib().fr_create(ctypes.byref(h), device, 0, N.FR_DTYPE_BF16), "fr_create")
            handle = h
        self._h = handle
        if x3_min_rows is not None:  # FR_OPT_X3_MIN_ROWS: smallest gallery given the bf16x3 path
            N.check(N.lib().fr_set_option(self._h, N.FR_OPT_X3_MIN_ROWS, int(x3_min_rows)), "fr_set_option")
        self._n = 0  # rows live on the device only (fr_gallery_write appends in place)
        N.check(N.lib().fr_gallery_set(self._h, None, 0, dim, self.index_base, 0), "fr_gallery_set")  # base, dim
        if rows is not None:
            self.add(rows)

    @property
    def ntotal(self) -> int:
        return self._n

    def reset(self) -> None:
        self._n = 0
        N.check(N.lib().fr_gallery_set(self._h, None, 0, self.d, self.index_base, 0), "fr_gallery_set")

    def _write(self, row0: int, rows) -> int:
        """fr_gallery_write of rows [row0, row0 + n) from host or device memory; returns n."""
        import torch

        r = rows if torch.is_tensor(rows) else torch.from_numpy(np.ascontiguousarray(np.asarray(rows, np.float32)))
        r = r.detach().float().reshape(-1, self.d).contiguous()
        n = int(r.shape[0])
        if n:
            N.check(N.lib().fr_gallery_write(self._h, N.ptr(r), int(row0), n, self.d, int(r.is_cuda)),
                    "fr_gallery_write")
        return n

    def add(self, rows) -> None:
        """Append rows (IndexFlatIP.add): written in place on the device, amortised O(new rows)."""
        self._n += self._write(self._n, rows)

    def update(self, row0: int, rows) -> None:
        """Overwrite rows [row0, row0 + n) (a dict-db entry re-embedded); row0 + n may run past the end."""
        if not 0 <= row0 <= self._n:
            raise IndexError(f"row {row0} outside a {self._n}-row gallery")
        self._n = max(self._n, row0 + self._write(row0, rows))

    def set_device_rows(self, rows_dev) -> None:
        """Install rows already resident on the GPU (no host round trip; the library copies them)."""
        rows_dev = rows_dev.float().contiguous()
        N.check(N.lib().fr_gallery_set(self._h, N.ptr(rows_dev), int(rows_dev.shape[0]), self.d, self.index_base, 1),
                "fr_gallery_set")
        self._n = int(rows_dev.shape[0])

    def set_exact(self, exact: bool) -> None:
        """FR_OPT_MATCH_EXACT: force the f32-MFMA kernel (default: bf16x3 candidates + exact rescoring
        for galleries of >= FR_OPT_X3_MIN_ROWS rows; both return the exact f32 top-k)."""
        N.check(N.lib().fr_set_option(self._h, N.FR_OPT_MATCH_EXACT, int(bool(exact))), "fr_set_option")

    def fallbacks(self) -> int:
        """Probes whose bf16x3 candidate proof failed and were rescanned exactly (device sync)."""
        return int(N.lib().fr_debug_match_fallbacks(self._h))

    def search_device(self, probes_dev, k: int, out_s=None, out_i=None):
        """probes_dev: cuda f32 [B, D] → (scores [B,k] f32, idx [B,k] int32) on the device, written into
        out_s / out_i when given (contiguous [B, k] f32 / int32 device tensors: no allocation)."""
        import torch

        p = probes_dev.float().contiguous()
        B = int(p.shape[0])
        s = out_s if out_s is not None else torch.empty((B, k), dtype=torch.float32, device=self.device)
        i = out_i if out_i is not None else torch.empty((B, k), dtype=torch.int32, device=self.device)
        if tuple(s.shape) != (B, k) or tuple(i.shape) != (B, k) or not (s.is_contiguous() and i.is_contiguous()) \
                or s.dtype != torch.float32 or i.dtype != torch.int32:
            raise ValueError(f"search_device: out_s / out_i must be contiguous [{B}, {k}] float32 / int32")
        N.check(N.lib().fr_match_topk(self._h, N.ptr(p), B, k, N.ptr(s), N.ptr(i), N.stream_ptr(self.device)),
                "fr_match_topk")
        return s, i

    def search(self, probes, k: int) -> Tuple[np.ndarray, np.ndarray]:
        """IndexFlatIP.search: (scores [B,k] f32, ids [B,k] int64, -1 where fewer than k rows)."""
        import torch

        p = torch.as_tensor(np.asarray(probes, dtype=np.float32) if not torch.is_tensor(probes) else probes)
        p = p.reshape(-1, self.d).to(self.device)
        if p.shape[0] == 0:
            return np.zeros((0, k), np.float32), np.zeros((0, k), np.int64)
        if self.ntotal == 0:
            B = p.shape[0]
            return np.full((B, k), -np.inf, np.float32), np.full((B, k), -1, np.int64)
        s, i = self.search_device(p, k)
        return s.cpu().numpy(), i.cpu().numpy().astype(np.int64)

    def close(self) -> None:
        if self._own and getattr(self, "_h", None):
            N.lib().fr_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
