"""Fused IResNet100 transition block layer1.0 (conv_trans.hip: conv1 3x3 + PReLU with its rows kept in LDS,
conv2 3x3/s2 + the K-concatenated downsample, one workgroup per image) vs the plan's member convs.

Both paths apply the same folded weights with the same bf16 / f16 rounding point (t is rounded once before
conv2); only the f32 summation order differs (the fused kernel sums the downsample first), so the block
output agrees to rounding noise and the embeddings to the stage tests' bar."""
import ctypes

import numpy as np
import pytest
import torch

from facerecognition_amd import _native as N

pytestmark = pytest.mark.gpu


def _tensor(m, B, name):
    L = N.lib()
    for t in range(L.fr_debug_tensor_count(m.handle)):
        if L.fr_debug_tensor_name(m.handle, t).decode() != name:
            continue
        dt = torch.float16 if L.fr_debug_tensor_dtype(m.handle, t) == N.FR_DTYPE_F16 else torch.bfloat16
        H, W, C = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        N.check(L.fr_debug_tensor_shape(m.handle, t, ctypes.byref(H), ctypes.byref(W), ctypes.byref(C)))
        buf = torch.empty((B, H.value, W.value, C.value), dtype=dt, device="cuda")
        N.check(L.fr_debug_copy_tensor(m.handle, t, B, buf.data_ptr(), N.stream_ptr()))
        torch.cuda.synchronize()
        return buf.float().cpu()
    raise KeyError(name)


def _plan(m, B):
    buf = ctypes.create_string_buffer(1 << 20)
    N.check(N.lib().fr_debug_plan(m.handle, B, buf, len(buf)), "fr_debug_plan")
    return buf.value.decode()


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("B", [1, 3, 9])
def test_trans_matches_member_convs(gpu, dtype, B):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("iresnet100", dtype=dtype)
    x = torch.from_numpy(synthetic_crops(B, 112, seed=11))
    m.set_option(N.FR_OPT_STAGE, 2)  # every fused kernel runs (auto would measure per batch size)
    assert "trans " in _plan(m, B)
    e_f = m.embed(x).cpu().numpy()
    y_f = _tensor(m, B, "layer1.0")
    m.set_option(N.FR_OPT_STAGE, 0)
    assert "trans " not in _plan(m, B)
    e_c = m.embed(x).cpu().numpy()
    y_c = _tensor(m, B, "layer1.0")
    m.close()
    rel = ((y_f - y_c).norm() / y_c.norm()).item()
    # t is rounded to 16 bits in both paths; a different f32 summation order flips a few of those roundings
    assert rel < (4e-3 if dtype == "bf16" else 5e-4), f"layer1.0: fused vs member convs rel err {rel:.3e}"
    cos = np.sum(e_f * e_c, axis=1)
    tol = 3e-4 if dtype == "bf16" else 5e-5
    assert np.all(1 - cos <= tol), f"fused vs member-conv embeddings: 1-cos = {1 - cos}"


def test_trans_full_batch_against_oracle(gpu):
    """bs = 256 (one image per CU: the batch the kernel is built for), fused kernel forced on: every face
    within the 1e-3 cosine bar of the fp32 oracle."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    from facerecognition_amd.weights import synth_state_dict
    from oracle import models as M
    B = 256
    m = FRModel.synthetic("iresnet100", max_batch=B)
    m.set_option(N.FR_OPT_STAGE, 2)
    u8 = synthetic_crops(B, 112, seed=21)
    e = m.embed(torch.from_numpy(u8)).cpu().numpy()
    assert "trans " in _plan(m, B)
    m.close()
    idx = np.arange(0, B, 32)  # an oracle sample (fp32 CPU forward)
    ref = M.embed(M.build_model("iresnet100", synth_state_dict("iresnet100")), "iresnet100", u8[idx])
    cos = np.sum(e[idx] * ref, axis=1) / (np.linalg.norm(e[idx], axis=1) * np.linalg.norm(ref, axis=1))
    assert np.all(1 - cos <= 1e-3), f"1-cos vs oracle {1 - cos}"
    assert np.all(np.isfinite(e))


def test_trans_graph_replay_repeatable(gpu):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("iresnet100")
    m.set_option(N.FR_OPT_STAGE, 2)
    x = torch.from_numpy(synthetic_crops(6, 112, seed=5)).cuda()
    outs = [m.embed(x).cpu().numpy() for _ in range(4)]
    m.close()
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])
