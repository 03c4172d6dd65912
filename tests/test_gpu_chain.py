"""FaceNet IRV1 repeat_2 as one launch (conv_chain.hip: the ten Block17 with the block input resident in LDS, one
workgroup per image) vs the plan's 40 member convs, and vs the fp32 oracle (reference: facenet_model.py:12-16 ->
facenet_pytorch InceptionResnetV1.repeat_2).

Both paths apply the same folded weights and round t1, t, b1, b0 and every block output to the storage format at
the same points; only the f32 summation order differs (the chain accumulates conv2d onto bias + x), so the
repeat_2 output agrees to rounding noise and the embeddings to the stage tests' bar."""
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
def test_chain_matches_member_convs(gpu, dtype, B):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("irv1_facenet", dtype=dtype)
    x = torch.from_numpy(synthetic_crops(B, 160, seed=13))
    m.set_option(N.FR_OPT_STAGE, 2)  # the chain runs (auto would measure per batch size)
    m.set_option(N.FR_OPT_FUSED_MASK, 8)  # ... and no other fused kernel before it
    assert "chain " in _plan(m, B)
    e_f = m.embed(x).cpu().numpy()
    mid_f = _tensor(m, B, "model.mixed_6a")
    y_f = _tensor(m, B, "model.repeat_2.9")
    m.set_option(N.FR_OPT_STAGE, 0)
    assert "chain " not in _plan(m, B)
    e_c = m.embed(x).cpu().numpy()
    mid_c = _tensor(m, B, "model.mixed_6a")
    y_c = _tensor(m, B, "model.repeat_2.9")
    m.close()
    assert torch.equal(mid_f, mid_c), "the chain's input differs: the runs are not comparable"
    rel_in = 0.0
    rel = ((y_f - y_c).norm() / y_c.norm()).item()
    # 50 roundings to 16 bits per element in both paths; a different f32 summation order flips a few of them
    assert rel < (6e-3 if dtype == "bf16" else 8e-4), f"repeat_2: chain vs member convs rel err {rel:.3e}"
    cos = np.sum(e_f * e_c, axis=1)
    tol = 3e-4 if dtype == "bf16" else 5e-5
    assert np.all(1 - cos <= tol), f"chain vs member-conv embeddings: 1-cos = {1 - cos}"
    print(f"{dtype} B={B}: mixed_6a rel {rel_in:.2e}, repeat_2 rel {rel:.2e}, max 1-cos {float((1 - cos).max()):.2e}")


def test_chain_full_batch_against_oracle(gpu):
    """bs = 256 (one image per CU), chain forced on: every sampled face within the 1e-3 cosine bar of the fp32
    oracle, and the same planted top-1 as the oracle embedding."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    from facerecognition_amd.weights import synth_state_dict
    from oracle import models as M
    B = 256
    m = FRModel.synthetic("irv1_facenet", max_batch=B)
    m.set_option(N.FR_OPT_STAGE, 2)
    u8 = synthetic_crops(B, 160, seed=23)
    e = m.embed(torch.from_numpy(u8)).cpu().numpy()
    assert "chain " in _plan(m, B)
    m.close()
    assert np.all(np.isfinite(e))
    idx = np.arange(0, B, 32)  # an oracle sample (fp32 CPU forward)
    ref = M.embed(M.build_model("irv1_facenet", synth_state_dict("irv1_facenet")), "irv1_facenet", u8[idx])
    cos = np.sum(e[idx] * ref, axis=1) / (np.linalg.norm(e[idx], axis=1) * np.linalg.norm(ref, axis=1))
    print(f"chain bs=256 vs oracle: max 1-cos {float((1 - cos).max()):.2e}")
    assert np.all(1 - cos <= 1e-3), f"1-cos vs oracle {1 - cos}"


def test_chain_graph_replay_repeatable(gpu):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("irv1_facenet")
    m.set_option(N.FR_OPT_STAGE, 2)
    x = torch.from_numpy(synthetic_crops(6, 160, seed=7)).cuda()
    outs = [m.embed(x).cpu().numpy() for _ in range(4)]
    m.close()
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])


# ---- the IRV1 stem as one launch (conv_stem160.hip: conv2d_1a .. conv2d_3b, row rings in LDS; with u8 crops it
# also prepares the input itself)
@pytest.mark.parametrize("fmt", ["u8", "f32"])
@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("B", [1, 3, 9])
def test_stem160_matches_member_ops(gpu, dtype, B, fmt):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("irv1_facenet", dtype=dtype)
    u8 = synthetic_crops(B, 160, seed=17)
    # f32: the reference transform's output (x / 255 - 0.5) / 0.5 in NCHW; the prepared-input path
    x = torch.from_numpy(u8) if fmt == "u8" else torch.from_numpy((u8.astype(np.float32) / 255 - 0.5) / 0.5).permute(0, 3, 1, 2).contiguous()
    m.set_option(N.FR_OPT_STAGE, 2)
    m.set_option(N.FR_OPT_FUSED_MASK, 2)
    assert "stem160 " in _plan(m, B)
    e_f = m.embed(x).cpu().numpy()
    e_f2 = m.embed(x).cpu().numpy()  # graph replay
    y_f = _tensor(m, B, "model.conv2d_3b")
    m.set_option(N.FR_OPT_STAGE, 0)
    assert "stem160 " not in _plan(m, B)
    e_c = m.embed(x).cpu().numpy()
    y_c = _tensor(m, B, "model.conv2d_3b")
    m.close()
    assert np.array_equal(e_f, e_f2)
    rel = ((y_f - y_c).norm() / y_c.norm()).item()
    cos = np.sum(e_f * e_c, axis=1)
    print(f"{dtype} {fmt} B={B}: conv2d_3b rel {rel:.2e}, max 1-cos {float((1 - cos).max()):.2e}")
    # a few f16 rounding flips from the different f32 summation order (4-5e-5 at maxpool_3a before 3b joined)
    assert rel < 3e-4, f"conv2d_3b: fused vs member ops rel err {rel:.3e}"
    # the stem is f16 in both plans; tiny stem differences grow through the network (more in the bf16 plan, whose
    # body from mixed_7a on is bf16)
    tol = 5e-4 if dtype == "bf16" else 5e-5
    assert np.all(1 - cos <= tol), f"fused stem vs member-op embeddings: 1-cos = {1 - cos}"


# ---- repeat_1 as one launch (conv_chain35.hip: five Block35, branch tensors in LDS, block outputs through global)
@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("B", [1, 3, 9])
def test_chain35_matches_member_convs(gpu, dtype, B):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("irv1_facenet", dtype=dtype)
    x = torch.from_numpy(synthetic_crops(B, 160, seed=19))
    m.set_option(N.FR_OPT_STAGE, 2)
    m.set_option(N.FR_OPT_FUSED_MASK, 4)
    assert " 256 300 300 5 " in _plan(m, B)
    e_f = m.embed(x).cpu().numpy()
    in_f = _tensor(m, B, "model.conv2d_4b")
    y_f = _tensor(m, B, "model.repeat_1.4")
    m.set_option(N.FR_OPT_STAGE, 0)
    e_c = m.embed(x).cpu().numpy()
    in_c = _tensor(m, B, "model.conv2d_4b")
    y_c = _tensor(m, B, "model.repeat_1.4")
    m.close()
    assert torch.equal(in_f, in_c), "the chain's input differs: the runs are not comparable"
    rel = ((y_f - y_c).norm() / y_c.norm()).item()
    cos = np.sum(e_f * e_c, axis=1)
    print(f"{dtype} B={B}: repeat_1 rel {rel:.2e}, max 1-cos {float((1 - cos).max()):.2e}")
    assert rel < (6e-3 if dtype == "bf16" else 1.5e-3), f"repeat_1: chain vs member convs rel err {rel:.3e}"
    # rounding-level differences at repeat_1 are amplified by the bf16 body after it (see the stem test)
    tol = 1e-3 if dtype == "bf16" else 5e-5
    assert np.all(1 - cos <= tol), f"chain35 vs member-conv embeddings: 1-cos = {1 - cos}"


# ---- ResNet-50 layer3.1 .. layer3.5 as one launch (conv_chain_r50.hip: five Bottlenecks at 7x7x1024, the block input
# resident in LDS; reference: arcface_model.py:118-132, the torchvision resnet50 backbone)
@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("B", [1, 3, 9])
def test_chain_r50_matches_member_convs(gpu, dtype, B):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("resnet50_arcface", dtype=dtype)
    x = torch.from_numpy(synthetic_crops(B, 112, seed=29))
    m.set_option(N.FR_OPT_STAGE, 2)
    m.set_option(N.FR_OPT_FUSED_MASK, 16)
    assert " 1024 1088 1088 5 " in _plan(m, B)
    e_f = m.embed(x).cpu().numpy()
    e_f2 = m.embed(x).cpu().numpy()  # graph replay
    in_f = _tensor(m, B, "backbone.layer3.0")
    y_f = _tensor(m, B, "backbone.layer3.5")
    m.set_option(N.FR_OPT_STAGE, 0)
    assert " 1024 1088 1088 5 " not in _plan(m, B)
    e_c = m.embed(x).cpu().numpy()
    in_c = _tensor(m, B, "backbone.layer3.0")
    y_c = _tensor(m, B, "backbone.layer3.5")
    m.close()
    assert np.array_equal(e_f, e_f2)
    assert torch.equal(in_f, in_c), "the chain's input differs: the runs are not comparable"
    rel = ((y_f - y_c).norm() / y_c.norm()).item()
    cos = np.sum(e_f * e_c, axis=1)
    print(f"{dtype} B={B}: layer3.5 rel {rel:.2e}, max 1-cos {float((1 - cos).max()):.2e}")
    # 15 roundings to 16 bits per element in both paths; a different f32 summation order flips a few of them
    assert rel < (6e-3 if dtype == "bf16" else 1.5e-3), f"layer3.5: chain vs member convs rel err {rel:.3e}"
    tol = 2e-4 if dtype == "bf16" else 2e-5
    assert np.all(1 - cos <= tol), f"chain_r50 vs member-conv embeddings: 1-cos = {1 - cos}"


def test_chain_r50_full_batch_against_oracle(gpu):
    """bs = 256 (one image per CU), the stem, layer1 Bottleneck and layer3 chain kernels forced on: sampled faces within the 1e-3 cosine bar of the fp32 oracle
    (the reference's own ResNet-50 ArcFace, golden-pinned in test_golden.py)."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    from facerecognition_amd.weights import synth_state_dict
    from oracle import models as M
    B = 256
    m = FRModel.synthetic("resnet50_arcface", max_batch=B)
    m.set_option(N.FR_OPT_STAGE, 2)
    u8 = synthetic_crops(B, 112, seed=31)
    e = m.embed(torch.from_numpy(u8)).cpu().numpy()
    plan = _plan(m, B)
    assert " 1024 1088 1088 5 " in plan and " 256 272 272 3 " in plan and " 64 392 392 1 " in plan
    m.close()
    assert np.all(np.isfinite(e))
    idx = np.arange(0, B, 32)
    ref = M.embed(M.build_model("resnet50_arcface", synth_state_dict("resnet50_arcface")), "resnet50_arcface", u8[idx])
    cos = np.sum(e[idx] * ref, axis=1) / (np.linalg.norm(e[idx], axis=1) * np.linalg.norm(ref, axis=1))
    print(f"chain_r50 bs=256 vs oracle: max 1-cos {float((1 - cos).max()):.2e}")
    assert np.all(1 - cos <= 1e-3), f"1-cos vs oracle {1 - cos}"


# ---- ResNet-50 layer1 (conv_bneck28.hip: one launch per Bottleneck at 28x28, one workgroup per image walking its rows;
# layer1.0 with its downsample K-concatenated into conv3; reference: arcface_model.py:118-132)
@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("B", [1, 3, 9])
def test_bneck28_matches_member_convs(gpu, dtype, B):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("resnet50_arcface", dtype=dtype)
    x = torch.from_numpy(synthetic_crops(B, 112, seed=37))
    m.set_option(N.FR_OPT_STAGE, 2)
    m.set_option(N.FR_OPT_FUSED_MASK, 32)
    assert " 256 272 272 3 " in _plan(m, B)
    e_f = m.embed(x).cpu().numpy()
    e_f2 = m.embed(x).cpu().numpy()  # graph replay
    in_f = _tensor(m, B, "backbone.maxpool")
    y0_f = _tensor(m, B, "backbone.layer1.0")
    y1_f = _tensor(m, B, "backbone.layer1.1")
    y_f = _tensor(m, B, "backbone.layer1.2")
    m.set_option(N.FR_OPT_STAGE, 0)
    assert " 256 272 272 3 " not in _plan(m, B)
    e_c = m.embed(x).cpu().numpy()
    in_c = _tensor(m, B, "backbone.maxpool")
    y0_c = _tensor(m, B, "backbone.layer1.0")
    y1_c = _tensor(m, B, "backbone.layer1.1")
    y_c = _tensor(m, B, "backbone.layer1.2")
    m.close()
    assert np.array_equal(e_f, e_f2)
    assert torch.equal(in_f, in_c), "the kernels' input differs: the runs are not comparable"
    rel0 = ((y0_f - y0_c).norm() / y0_c.norm()).item()
    rel1 = ((y1_f - y1_c).norm() / y1_c.norm()).item()
    rel = ((y_f - y_c).norm() / y_c.norm()).item()
    cos = np.sum(e_f * e_c, axis=1)
    print(f"{dtype} B={B}: layer1.0 rel {rel0:.2e}, layer1.1 rel {rel1:.2e}, layer1.2 rel {rel:.2e}, "
          f"max 1-cos {float((1 - cos).max()):.2e}")
    # 3 roundings to 16 bits per block in both paths; only the f32 summation order differs
    assert rel0 < (3e-3 if dtype == "bf16" else 7e-4), f"layer1.0: kernel vs member convs rel err {rel0:.3e}"
    assert rel1 < (4e-3 if dtype == "bf16" else 1e-3), f"layer1.1: kernel vs member convs rel err {rel1:.3e}"
    assert rel < (6e-3 if dtype == "bf16" else 1.5e-3), f"layer1.2: kernel vs member convs rel err {rel:.3e}"
    # three blocks of flipped bf16 roundings carried through the 13 blocks after them (the oracle bar is 1e-3)
    tol = 4e-4 if dtype == "bf16" else 2e-5
    assert np.all(1 - cos <= tol), f"bneck28 vs member-conv embeddings: 1-cos = {1 - cos}"


# ---- ResNet-50 stem (conv_stem_r50.hip: conv1 7x7/s2 + ReLU + maxpool 3x3/s2 in one launch, one workgroup per image;
# reference: arcface_model.py:118-132, the torchvision resnet50 stem)
@pytest.mark.parametrize("fmt", ["u8", "f32"])
@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("B", [1, 3, 9])
def test_stem_r50_matches_member_ops(gpu, dtype, B, fmt):
    """u8 crops: the kernel prepares them itself (no preprocess launch); f32 (the reference transform's output in
    NCHW): the kernel reads the prepared tensor."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("resnet50_arcface", dtype=dtype)
    u8 = synthetic_crops(B, 112, seed=41)
    x = torch.from_numpy(u8) if fmt == "u8" else \
        torch.from_numpy((u8.astype(np.float32) / 255 - 0.5) / 0.5).permute(0, 3, 1, 2).contiguous()
    m.set_option(N.FR_OPT_STAGE, 2)
    m.set_option(N.FR_OPT_FUSED_MASK, 64)
    assert " 64 392 392 1 " in _plan(m, B)
    e_f = m.embed(x).cpu().numpy()
    e_f2 = m.embed(x).cpu().numpy()  # graph replay
    y_f = _tensor(m, B, "backbone.maxpool")
    m.set_option(N.FR_OPT_STAGE, 0)
    assert " 64 392 392 1 " not in _plan(m, B)
    e_c = m.embed(x).cpu().numpy()
    y_c = _tensor(m, B, "backbone.maxpool")
    m.close()
    assert np.array_equal(e_f, e_f2)
    rel = ((y_f - y_c).norm() / y_c.norm()).item()
    cos = np.sum(e_f * e_c, axis=1)
    print(f"{dtype} {fmt} B={B}: maxpool rel {rel:.2e}, max 1-cos {float((1 - cos).max()):.2e}")
    # one rounding to 16 bits (the conv output) in both paths; only the conv's f32 summation order differs
    assert rel < (2e-3 if dtype == "bf16" else 3e-4), f"stem: kernel vs member ops rel err {rel:.3e}"
    tol = 3e-4 if dtype == "bf16" else 2e-5
    assert np.all(1 - cos <= tol), f"stem_r50 vs member-op embeddings: 1-cos = {1 - cos}"
