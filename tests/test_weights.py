"""Weight folding on the CPU (facerecognition_amd/weights.py): every fold is an algebraic identity of
the reference modules in eval mode, checked here in f64/f32 against the unfolded torch ops."""
import numpy as np
import torch

from facerecognition_amd import weights as W


def _cls(H, Wd):
    rc = np.ones(H, int)
    rc[0], rc[-1] = 0, 2
    cc = np.ones(Wd, int)
    cc[0], cc[-1] = 0, 2
    return 3 * rc[:, None] + cc[None, :]


def test_pre_conv_bn_fold_border_classes():
    """bn2(conv(pad0(bn1(x)))) == conv(pad0(x), w') + b9[border class] (IBasicBlock conv1)."""
    rng = np.random.default_rng(0)
    O, C = 6, 5
    w = rng.standard_normal((O, 3, 3, C))
    s1, t1 = rng.uniform(.5, 1.5, C), rng.standard_normal(C)
    s2, t2 = rng.uniform(.5, 1.5, O), rng.standard_normal(O)
    out = {}
    W._fold_pre_bn_3x3(out, "c", w, s1, t1, s2, t2, np.zeros(O))
    assert out["c.b9"].shape == (9, O) and np.array_equal(out["c.b"], out["c.b9"][4])
    for H, Wd in ((7, 7), (3, 5), (14, 14)):
        x = torch.tensor(rng.standard_normal((2, C, H, Wd)))
        wt = torch.tensor(w).permute(0, 3, 1, 2)
        ref = torch.nn.functional.conv2d(x * torch.tensor(s1)[None, :, None, None]
                                         + torch.tensor(t1)[None, :, None, None], wt, padding=1)
        ref = ref * torch.tensor(s2)[None, :, None, None] + torch.tensor(t2)[None, :, None, None]
        got = torch.nn.functional.conv2d(x, torch.tensor(out["c.w"].astype(np.float64)).permute(0, 3, 1, 2),
                                         padding=1)
        got = got + torch.tensor(out["c.b9"].astype(np.float64))[torch.tensor(_cls(H, Wd))].permute(2, 0, 1)[None]
        assert (got - ref).abs().max().item() < 1e-5


def test_iresnet100_fold_matches_module_algebra():
    """Folded IResNet100 tensors reproduce the oracle's block conv1 / conv2 and head on random inputs."""
    from oracle import models as M
    sd = W.synth_state_dict("iresnet100", seed=3, calibrated=False)
    f = W.fold_state_dict("iresnet100", sd)
    om = M.build_model("iresnet100", sd).double()
    blk = om.layer2[1]
    x = torch.randn(1, 128, 28, 28, dtype=torch.float64)
    with torch.no_grad():
        ref = blk.prelu(blk.bn2(blk.conv1(blk.bn1(x))))
    w = torch.tensor(f["layer2.1.conv1.w"].astype(np.float64)).permute(0, 3, 1, 2)
    got = torch.nn.functional.conv2d(x, w, padding=1)
    got = got + torch.tensor(f["layer2.1.conv1.b9"].astype(np.float64))[torch.tensor(_cls(28, 28))].permute(2, 0, 1)[None]
    got = torch.nn.functional.prelu(got, torch.tensor(f["layer2.1.conv1.slope"].astype(np.float64)))
    assert ((got - ref).norm() / ref.norm()).item() < 1e-5
    with torch.no_grad():
        ref2 = blk.bn3(blk.conv2(ref))
    w2 = torch.tensor(f["layer2.1.conv2.w"].astype(np.float64)).permute(0, 3, 1, 2)
    got2 = torch.nn.functional.conv2d(ref, w2, padding=1) + torch.tensor(f["layer2.1.conv2.b"].astype(np.float64))[None, :, None, None]
    assert ((got2 - ref2).norm() / ref2.norm()).item() < 1e-5
    # no producer writes a bn1 copy any more
    assert not any(k.endswith(".bn1.s") for k in f)


def test_resnet50_head_fold():
    sd = W.synth_state_dict("resnet50_arcface", seed=2, num_classes=10, calibrated=False)
    f = W.fold_state_dict("resnet50_arcface", sd)
    from oracle import models as M
    om = M.build_model("resnet50_arcface", sd, num_classes=10).double()
    feat = torch.randn(3, 2048, dtype=torch.float64)
    with torch.no_grad():
        ref = om.bn2(om.fc(om.bn1(feat)))
    got = feat @ torch.tensor(f["head.w"].astype(np.float64)).T + torch.tensor(f["head.b"].astype(np.float64))
    assert ((got - ref).norm() / ref.norm()).item() < 1e-5


def test_blob_round_trip_sizes():
    f = W.fold_state_dict("iresnet100", W.synth_state_dict("iresnet100", seed=1, calibrated=False))
    blob = W.pack_blob(f)
    assert blob[:4] == b"FRW1" and int.from_bytes(blob[4:8], "little") == len(f)


def test_facenet_projection_fold_and_oracle():
    """FaceNetModel(embedding_size=128): projection.{weight,bias} pass through as proj.{w,b}; the oracle
    builds the projection from the state_dict (facenet_model.py:20-23,32-35)."""
    from oracle import models as M
    sd = W.synth_state_dict("irv1_facenet", embedding_size=128)
    out = W.fold_state_dict("irv1_facenet", sd)
    assert out["proj.w"].shape == (128, 512) and out["proj.b"].shape == (128,)
    np.testing.assert_array_equal(out["proj.w"], sd["projection.weight"])
    m = M.build_model("irv1_facenet", sd)
    assert m.projection is not None and m.projection.out_features == 128
    x = torch.randn(3, 512)
    e = torch.nn.functional.normalize(x, dim=1)
    ref = torch.nn.functional.normalize(m.projection(e), dim=1)
    got = torch.nn.functional.normalize(e @ torch.tensor(out["proj.w"]).T + torch.tensor(out["proj.b"]), dim=1)
    assert torch.allclose(got, ref, atol=1e-6)


def test_quantize_fp8_weights():
    """quantize_fp8: per-output-channel scale = max|w| / 448, values e4m3-representable, dequant error
    within half an e4m3 ulp (2^-4 relative for normals), stem and head untouched."""
    sd = W.synth_state_dict("iresnet100")
    f = W.fold_state_dict("iresnet100", sd)
    q = W.quantize_fp8(f)
    assert "conv1.wscale" not in q and "head.wscale" not in q
    k = "layer3.5.conv2"
    w, qw, s = f[k + ".w"], q[k + ".w"], q[k + ".wscale"]
    assert s.shape == (w.shape[0],) and np.allclose(s, np.abs(w).reshape(w.shape[0], -1).max(1) / 448)
    rt = torch.from_numpy(qw).to(torch.float8_e4m3fn).float().numpy()
    assert np.array_equal(rt, qw)                       # exactly representable
    assert np.abs(qw).max() <= 448
    deq = qw * s[:, None, None, None]
    # half an ulp: 2^-4 relative for normals, 2^-10 (scaled) absolute in the subnormal range
    bound = 2 ** -4 * np.abs(w) + 2 ** -10 * s[:, None, None, None] * (1 + 1e-5)
    assert np.all(np.abs(deq - w) <= bound + 1e-12)
