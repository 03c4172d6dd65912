"""Batch-size (in)dependence of the embeddings (reference recognition_engine.py:383-389, where
recognize_batch is a loop over recognize, so a face gets the same result in any batch).

* FR_OPT_BATCH_INVARIANT (the RecognitionEngine's default): every kernel sums K in the implicit GEMM's order and
  the head keeps one split plan, so a face's embedding is the same bits at bs = 1, 9 and 64.
* The default throughput mode measures the fastest kernels per batch size (LDS-resident stages, the fused
  transition, split-K, small-M kernels); their f32 summation orders differ.  The drift between batch sizes is
  measured here and printed; the bound asserted is the north star's 1e-3 cosine (the measured values are far below
  it)."""
import ctypes

import numpy as np
import pytest
import torch

from facerecognition_amd import _native as N

pytestmark = pytest.mark.gpu


def _plan(m, B):
    buf = ctypes.create_string_buffer(1 << 20)
    N.check(N.lib().fr_debug_plan(m.handle, B, buf, len(buf)), "fr_debug_plan")
    return buf.value.decode()


def _embed_in_chunks(m, x, bs):
    return np.concatenate([m.embed(x[i:i + bs]).cpu().numpy() for i in range(0, len(x), bs)])


@pytest.mark.parametrize("arch", ["iresnet100", "irv1_facenet", "resnet50_arcface"])
def test_invariant_mode_is_bitwise_batch_independent(gpu, arch):
    """bs = 256 (the bench batch, where the tuner sees the largest M and may pick the 3-stage, 256x128, 128x256,
    register-ring or direct kernels) against bs = 64, 9 and 1 (small-M kernels): the same bits in invariant mode."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic(arch, max_batch=256)
    m.set_option(N.FR_OPT_BATCH_INVARIANT, 1)
    x = torch.from_numpy(synthetic_crops(256, m.input_size, seed=31)).cuda()
    e256 = m.embed(x).cpu().numpy()
    for B in (256, 64):
        plan = _plan(m, B)
        assert not any(l.split()[0] in ("stage", "stage8", "trans", "block", "chain", "stem160")
                       for l in plan.splitlines() if l.strip()), plan
    e64 = m.embed(x[:64]).cpu().numpy()
    e9 = _embed_in_chunks(m, x[:18], 9)
    e1 = _embed_in_chunks(m, x[:4], 1)
    m.close()
    assert np.array_equal(e64, e256[:64]), "bs = 64 vs bs = 256 differ in invariant mode"
    assert np.array_equal(e9, e256[:18]), "bs = 9 vs bs = 256 differ in invariant mode"
    assert np.array_equal(e1, e256[:4]), "bs = 1 vs bs = 256 differ in invariant mode"


def test_invariant_mode_refused_on_fp8(gpu):
    """fp8 handles scale their e4m3 convs' activations by a per-batch amax: the option is refused, and
    the engine leaves such a model in its default mode."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.recognition_engine import RecognitionEngine
    m = FRModel.synthetic("iresnet100", dtype="fp8", max_batch=8)
    with pytest.raises(RuntimeError, match="FP8"):
        m.set_option(N.FR_OPT_BATCH_INVARIANT, 1)
    assert m.get_option(N.FR_OPT_BATCH_INVARIANT) == 0
    RecognitionEngine(model_path=None, use_face_detection=False, model=m, batch_invariant=True)
    assert m.get_option(N.FR_OPT_BATCH_INVARIANT) == 0
    m.close()


def test_default_mode_batch_drift_measured(gpu):
    """Default (throughput) mode: the same faces embedded at bs = 256, 64, 9, 4 and 1; every batch size picks its
    own kernels.  Prints the max 1 - cos against bs = 256 per batch size."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    B = 256
    m = FRModel.synthetic("iresnet100", max_batch=B)
    x = torch.from_numpy(synthetic_crops(B, 112, seed=33)).cuda()
    ref = m.embed(x).cpu().numpy()
    worst = {}
    for bs, n in ((64, 128), (9, 36), (4, 16), (1, 8)):
        e = _embed_in_chunks(m, x[:n], bs)
        cos = np.sum(e * ref[:n], axis=1) / (np.linalg.norm(e, axis=1) * np.linalg.norm(ref[:n], axis=1))
        worst[bs] = float((1 - cos).max())
    m.close()
    print("max 1-cos vs bs=256 by batch size:", {k: f"{v:.2e}" for k, v in worst.items()})
    assert all(v <= 1e-3 for v in worst.values()), worst


def test_large_batch_runs_in_chunks(gpu):
    """A call above the engine's chunk size (every activation tensor < 2 GiB: 1280 faces for IResNet100, whose
    layer1 tensor is 1.6 MB per face) runs as several forwards: the faces past the first chunk get the same bits
    as when embedded on their own (invariant mode).  Before r05 a 2000-face call read layer1 past the kernels'
    2 GiB buffer range, and those faces got garbage."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("iresnet100", max_batch=64)
    m.set_option(N.FR_OPT_BATCH_INVARIANT, 1)
    x = torch.from_numpy(synthetic_crops(1300, 112, seed=35)).cuda()
    big = m.embed(x).cpu().numpy()
    tail = m.embed(x[1270:]).cpu().numpy()
    head = m.embed(x[:8]).cpu().numpy()
    m.close()
    assert np.isfinite(big).all()
    assert np.array_equal(big[1270:], tail)
    assert np.array_equal(big[:8], head)
