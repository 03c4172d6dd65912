"""``FRModel`` — the native backbone behind the reference's ``model(x, labels=None)`` boundary.

The reference calls ``model(img_tensor, labels=None)`` (ArcFace) or ``model(img_tensor)``
(FaceNet) and then ``F.normalize`` (inference/extract_embeddings.py:377-382, :430-435).
``FRModel`` keeps that call shape but runs the whole forward in libfrhip.so on the MI355X
(one C-ABI call, PyTorch-ROCm tensors in, device f32 embeddings out).  It accepts either the
reference's normalized f32 NCHW batch or aligned u8 NHWC crops (the north-star input), in
which case ToTensor+Normalize are fused into the first kernel.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _native as N
from . import weights as Wt


class FRModel:
    def __init__(self, arch: str, state_dict=None, device: int = 0, max_batch: int = 0, dtype: Optional[str] = None):
        import torch

        if arch not in Wt.ARCHS:
            raise ValueError(f"unknown arch {arch!r}")
        if not torch.cuda.is_available():
            raise RuntimeError("FRModel needs a ROCm GPU (torch.cuda.is_available() is False); "
                               "there is deliberately no CPU fallback")
        self.arch = arch
        self.dtype = dtype or Wt.DEFAULT_DTYPE[arch]
        if self.dtype not in N.FR_DTYPE:
            raise ValueError(f"dtype must be one of {sorted(N.FR_DTYPE)}, got {self.dtype!r}")
        self.device = torch.device("cuda", device)
        self.input_size = Wt.INPUT_SIZE[arch]
        L = N.lib()
        h = ctypes.c_void_p()
        N.check(L.fr_create(ctypes.byref(h), device, N.FR_ARCH[arch], N.FR_DTYPE[self.dtype]), "fr_create")
        self._h = h
        self.embedding_size = 512
        if state_dict is not None:
            self.load_state_dict(state_dict)
        if max_batch:
            self.reserve(max_batch)

    # -- construction helpers -------------------------------------------------------
    @classmethod
    def synthetic(cls, arch: str, seed: int = 1234, device: int = 0, max_batch: int = 0,
                  dtype: Optional[str] = None) -> "FRModel":
        return cls(arch, Wt.synth_state_dict(arch, seed=seed), device=device, max_batch=max_batch, dtype=dtype)

    @classmethod
    def from_checkpoint(cls, path: str, device: int = 0, dtype: Optional[str] = None) -> "FRModel":
        sd, _ = Wt.load_checkpoint(path)
        return cls(Wt.detect_arch(sd), sd, device=device, dtype=dtype)

    def load_state_dict(self, state_dict, strict: bool = True) -> None:
        folded = Wt.fold_state_dict(self.arch, state_dict)
        if self.dtype == "fp8":
            folded = Wt.quantize_fp8(folded, convs=Wt.fp8_plan(self.arch))
        blob = Wt.pack_blob(folded)
        buf = ctypes.create_string_buffer(blob, len(blob))
        N.check(N.lib().fr_load_weights(self._h, buf, len(blob)), "fr_load_weights")
        self.embedding_size = N.lib().fr_embed_dim(self._h)

    def set_option(self, option: int, value: int) -> None:
        """fr_set_option (FR_OPT_STAGE, FR_OPT_KEEP_INTERMEDIATES; include/frhip.h)."""
        N.check(N.lib().fr_set_option(self._h, int(option), int(value)), "fr_set_option")

    def get_option(self, option: int) -> int:
        return int(N.lib().fr_get_option(self._h, int(option)))

    def reserve(self, max_batch: int) -> None:
        N.check(N.lib().fr_reserve(self._h, int(max_batch)), "fr_reserve")

    # -- torch.nn.Module-compatible no-ops -----------------------------------------
    def eval(self):
        return self

    def to(self, *_a, **_k):
        return self

    # -- forward ---------------------------------------------------------------------
    def _prep(self, x):
        import torch

        if isinstance(x, np.ndarray):
            x = torch.from_numpy(x)
        if x.dtype == torch.uint8:
            if x.dim() != 4 or x.shape[-1] != 3:
                raise ValueError(f"u8 input must be NHWC [B,H,W,3], got {tuple(x.shape)}")
            fmt, H, W = N.FR_IN_U8_NHWC, x.shape[1], x.shape[2]
        else:
            if x.dim() != 4 or x.shape[1] != 3:
                raise ValueError(f"float input must be NCHW [B,3,H,W], got {tuple(x.shape)}")
            x = x.float()
            fmt, H, W = N.FR_IN_F32_NCHW, x.shape[2], x.shape[3]
        x = x.to(self.device, non_blocking=True).contiguous()
        return x, fmt, int(H), int(W)

    def embed(self, x, normalize: bool = True, out=None, sync: bool = True):
        """Device f32 [B, 512] embeddings (L2-normalized unless normalize=False).

        sync=True (default): a forward that ran an IResNet100 split stage is waited for and re-run on
        the per-conv path if a split-stage wait ran out, so the result is always valid.  sync=False
        (FR_EMBED_ASYNC, pipelined callers such as bench.py): returns once enqueued; a run-out wait
        leaves that image's embedding NaN and is reported by sync_check() / the next embed()."""
        import torch

        x, fmt, H, W = self._prep(x)
        B = int(x.shape[0])
        if out is None:
            out = torch.empty((B, self.embedding_size), dtype=torch.float32, device=self.device)
        flags = (0 if normalize else N.FR_EMBED_RAW) | (0 if sync else N.FR_EMBED_ASYNC)
        N.check(N.lib().fr_embed(self._h, N.ptr(x), fmt, B, H, W, N.ptr(out), flags, N.stream_ptr(self.device)),
                "fr_embed")
        return out

    def sync_check(self) -> None:
        """Synchronize the current stream; raise if an async forward's split-stage wait ran out."""
        N.check(N.lib().fr_sync_check(self._h, N.stream_ptr(self.device)), "fr_sync_check")

    def stage_timeouts(self) -> int:
        """Split-stage waits that ran out on this handle (fr_debug_stage_timeouts; 0 when healthy)."""
        return int(N.lib().fr_debug_stage_timeouts(self._h))

    def stage_reruns(self) -> int:
        """Forwards re-run on the per-conv path after a run-out wait (fr_debug_stage_reruns)."""
        return int(N.lib().fr_debug_stage_reruns(self._h))

    def __call__(self, x, labels=None):
        """Reference semantics: ArcFaceModel(x, labels=None) returns the un-normalized embedding;
        FaceNetModel(x) returns the normalized one (facenet_model.py:28-36)."""
        if labels is not None:
            raise NotImplementedError("training forward (ArcMarginProduct) is out of scope")
        return self.embed(x, normalize=(self.arch == "irv1_facenet"))

    forward = __call__

    def extract_features(self, x, normalize: bool = True):
        """ArcFaceModel.extract_features (arcface_model.py:204-217)."""
        return self.embed(x, normalize=normalize)

    def get_embedding_dim(self) -> int:
        return self.embedding_size

    def close(self) -> None:
        if getattr(self, "_h", None):
            N.lib().fr_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h
