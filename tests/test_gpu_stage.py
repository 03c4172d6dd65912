"""LDS-resident layer3 stage kernel (conv_stage.hip) vs the per-conv launch path of the same plan.

Both paths run the same folded ops with the same bf16/f16 rounding points; only the f32
accumulation order inside each conv differs, so the stage output must agree with the per-conv
path to within accumulation-order noise, and both stay at the 1e-3 cosine bar against the oracle
(tests/test_gpu_models.py runs with the stage on, its default)."""
import numpy as np
import pytest
import torch

from facerecognition_amd import _native as N

pytestmark = pytest.mark.gpu


def _named(m, B, names):
    import ctypes
    L = N.lib()
    dt = torch.float16 if m.dtype == "f16" else torch.bfloat16
    out = {}
    for t in range(L.fr_debug_tensor_count(m.handle)):
        name = L.fr_debug_tensor_name(m.handle, t).decode()
        if name not in names:
            continue
        H, W, C = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        N.check(L.fr_debug_tensor_shape(m.handle, t, ctypes.byref(H), ctypes.byref(W), ctypes.byref(C)))
        buf = torch.empty((B, H.value, W.value, C.value), dtype=dt, device="cuda")
        N.check(L.fr_debug_copy_tensor(m.handle, t, B, buf.data_ptr(), N.stream_ptr()))
        torch.cuda.synchronize()
        out[name] = buf.float().cpu()
    return out


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("B", [1, 5])
def test_stage_matches_per_conv_path(gpu, dtype, B):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("iresnet100", dtype=dtype)
    assert m.get_option(N.FR_OPT_STAGE) == 1
    x = torch.from_numpy(synthetic_crops(B, 112, seed=3))
    names = {"layer3.1.prelu", "layer3.1", "layer3.15", "layer3.29"}
    m.set_option(N.FR_OPT_KEEP_INTERMEDIATES, 1)
    m.set_option(N.FR_OPT_STAGE, 1)
    e_stage = m.embed(x).cpu().numpy()
    t_stage = _named(m, B, names)
    m.set_option(N.FR_OPT_STAGE, 0)
    e_conv = m.embed(x).cpu().numpy()
    t_conv = _named(m, B, names)
    m.close()
    cos = np.sum(e_stage * e_conv, axis=1)
    # a different f32 summation order flips some bf16 roundings; through 58 convs that is ~1e-4 cosine
    tol = 3e-4 if dtype == "bf16" else 5e-5
    assert np.all(1 - cos <= tol), f"stage vs per-conv embeddings: 1-cos = {1 - cos}"
    for n in sorted(names):
        a, b = t_stage[n], t_conv[n]
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert rel < 2e-2, f"{n}: stage vs per-conv rel err {rel:.3e}"


def test_stage_repeat_and_graph_replay(gpu):
    """Graph replays of the stage plan are bit-identical run to run (the stage buffer is in place)."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("iresnet100")
    x = torch.from_numpy(synthetic_crops(4, 112, seed=5)).cuda()
    outs = [m.embed(x).cpu().numpy() for _ in range(4)]
    m.close()
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])


def test_stage_absent_for_other_archs(gpu):
    from facerecognition_amd.model import FRModel
    m = FRModel.synthetic("resnet50_arcface")
    assert m.get_option(N.FR_OPT_STAGE) == 0
    m.close()
