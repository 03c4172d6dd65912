"""LDS-resident stage kernels -- layer3 (conv_stage.hip, one workgroup per image) and the layer2 / layer1
split stages (conv_split_stage.hip, two / four workgroups per image exchanging boundary rows per conv) --
vs the per-conv launch path of the same plan.

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
    out = {}
    for t in range(L.fr_debug_tensor_count(m.handle)):
        name = L.fr_debug_tensor_name(m.handle, t).decode()
        if name not in names:
            continue
        dt = torch.float16 if L.fr_debug_tensor_dtype(m.handle, t) == N.FR_DTYPE_F16 else torch.bfloat16
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
    # layer4.0.prelu / layer3.0.prelu: the layer3 / layer2 stages' tails (the next conv computed on the stage's
    # final patch)
    names = {"layer3.1.prelu", "layer3.1", "layer3.15", "layer3.29", "layer4.0.prelu", "layer2.1.prelu", "layer2.1",
             "layer2.6", "layer2.12", "layer3.0.prelu", "layer1.1.prelu", "layer1.1", "layer1.2"}
    m.set_option(N.FR_OPT_KEEP_INTERMEDIATES, 1)
    m.set_option(N.FR_OPT_STAGE, 2)  # always (auto would pick the per-conv path at these batch sizes)
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


def test_stage_auto_rule_by_batch(gpu):
    """Auto mode runs the stage kernel at every batch of at most one image per CU, and above that only
    when the CU rounds are >= 80 % full; the plan dump names what runs."""
    import ctypes
    from facerecognition_amd.model import FRModel
    m = FRModel.synthetic("iresnet100")
    L = N.lib()
    cu = torch.cuda.get_device_properties(0).multi_processor_count

    def has_stage(B, last="layer3.29"):
        buf = ctypes.create_string_buffer(1 << 16)
        N.check(L.fr_debug_plan(m.handle, B, buf, len(buf)), "fr_debug_plan")
        return any(l.startswith("stage") and l.endswith(last) for l in buf.value.decode().splitlines())

    assert has_stage(1) and has_stage(cu // 2) and has_stage(cu) and has_stage(2 * cu)
    assert not has_stage(cu + 1) and has_stage(2 * cu - cu // 8)
    # split stages: the same rule over rounds of cu / parts images (layer2: 2 parts, layer1: 4)
    def rule(B, parts):
        cap = cu // parts
        rounds = -(-B // cap)
        return B <= cap or B * 100 >= 80 * rounds * cap

    for B in (1, cu // 4, cu // 4 + 1, cu // 2 + 1, cu, cu + 1, 2 * cu - cu // 8):
        assert has_stage(B, "layer2.12") == rule(B, 2), B
        assert has_stage(B, "layer1.2") == rule(B, 4), B
    m.set_option(N.FR_OPT_STAGE_MIN_FILL, 0)
    assert has_stage(cu + 1)
    m.set_option(N.FR_OPT_STAGE_MIN_FILL, 80)
    m.set_option(N.FR_OPT_STAGE, 2)
    assert has_stage(cu + 1)
    m.set_option(N.FR_OPT_STAGE, 0)
    assert not has_stage(cu)
    # B = 257: the per-conv path (auto) gives the same embeddings as the forced stage path
    from facerecognition_amd.synthetic import synthetic_crops
    x = torch.from_numpy(synthetic_crops(cu + 1, 112, seed=9))
    m.set_option(N.FR_OPT_STAGE, 1)
    a = m.embed(x).cpu().numpy()
    m.set_option(N.FR_OPT_STAGE, 2)
    b = m.embed(x).cpu().numpy()
    m.close()
    assert np.all(1 - (a * b).sum(1) <= 3e-4)


def test_stage_absent_for_other_archs(gpu):
    """ResNet-50 gets none of IResNet100's LDS-resident stages or fused transition; its fused launches (round 6:
    the stem, conv_stem_r50.hip; layer1, conv_bneck28.hip; the layer3.1-3.5 chain, conv_chain_r50.hip) are governed
    by the stage option like the others."""
    import ctypes
    from facerecognition_amd.model import FRModel
    m = FRModel.synthetic("resnet50_arcface")
    assert m.get_option(N.FR_OPT_STAGE) == 1
    m.set_option(N.FR_OPT_STAGE, 2)
    buf = ctypes.create_string_buffer(1 << 20)
    N.check(N.lib().fr_debug_plan(m.handle, 256, buf, len(buf)), "fr_debug_plan")
    lines = buf.value.decode().splitlines()
    m.close()
    assert not [ln for ln in lines if ln.split()[0] in ("stage", "stage8", "trans", "stem160")]
    for sig in (" 1024 1088 1088 5 ", " 256 272 272 3 ", " 64 392 392 1 "):
        assert [ln for ln in lines if ln.startswith("chain ") and sig in ln], sig


SPLIT_CASES = [("layer2.12", "layer2.1.prelu", 2, B) for B in (1, 3, 17, 130)] + \
              [("layer1.2", "layer1.1.prelu", 4, B) for B in (1, 5, 70)]


@pytest.mark.parametrize("last,first_t,parts,B", SPLIT_CASES)
def test_split_stage_batches_and_exchange(gpu, last, first_t, parts, B):
    """Split stages at batch sizes that leave padded workgroup groups (B = 1, 3, 5, 17) and that span two
    rounds of CUs (B = 130 > 256 CUs / 2 for layer2, B = 70 > 256 / 4 for layer1): the stage's output
    agrees with the per-conv path image by image and part by part (a lost or stale boundary row shows up
    as a localized error in its part), and no bounded wait of the row exchange ran out."""
    import ctypes
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("iresnet100")
    L = N.lib()
    x = torch.from_numpy(synthetic_crops(B, 112, seed=40 + B))
    m.set_option(N.FR_OPT_KEEP_INTERMEDIATES, 1)
    m.set_option(N.FR_OPT_STAGE, 2)
    buf = ctypes.create_string_buffer(1 << 16)
    N.check(L.fr_debug_plan(m.handle, B, buf, len(buf)), "fr_debug_plan")
    assert any(l.startswith("stage") and l.endswith(last) for l in buf.value.decode().splitlines())
    e_stage = m.embed(x).cpu().numpy()
    t_stage = _named(m, B, {last, first_t})
    assert L.fr_debug_stage_timeouts(m.handle) == 0
    m.set_option(N.FR_OPT_STAGE, 0)
    e_conv = m.embed(x).cpu().numpy()
    t_conv = _named(m, B, {last, first_t})
    m.close()
    for n in t_stage:
        a, b = t_stage[n], t_conv[n]
        for i in range(B):  # per image and per part (14 rows each)
            for p in range(parts):
                r = slice(14 * p, 14 * p + 14)
                d = (a[i, r] - b[i, r]).norm() / (b[i, r].norm() + 1e-12)
                assert d < 2e-2, f"{n} image {i} rows {r}: rel err {d:.3e}"
    assert np.all(1 - np.sum(e_stage * e_conv, axis=1) <= 3e-4)


def test_split_stage_wait_runout_never_returns_valid_looking_embeddings(gpu):
    """A split-stage halo wait that runs out (FR_OPT_STAGE_SPIN_LIMIT < 0 forces every wait to) is never
    returned as a valid embedding: fr_embed's default waits for the forward and re-runs it on the
    per-conv path (correct results, fr_debug_stage_reruns), and FR_EMBED_ASYNC leaves the affected
    embeddings NaN and latches FR_ERR_STAGE, reported once by fr_sync_check or the next fr_embed."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("iresnet100")
    x = torch.from_numpy(synthetic_crops(6, 112, seed=77)).cuda()
    m.set_option(N.FR_OPT_STAGE, 2)
    good = m.embed(x).cpu().numpy()
    assert m.stage_timeouts() == 0 and m.stage_reruns() == 0
    m.set_option(N.FR_OPT_STAGE_SPIN_LIMIT, -1)
    e = m.embed(x).cpu().numpy()  # synchronous: detected and re-run without split stages
    assert m.stage_timeouts() > 0 and m.stage_reruns() == 1
    assert np.all(np.isfinite(e)) and np.all(1 - np.sum(e * good, axis=1) <= 3e-4)
    e2 = m.embed(x, sync=False)  # asynchronous: NaN embeddings + a latched error
    with pytest.raises(RuntimeError, match=r"rc=-6"):
        m.sync_check()
    assert bool(torch.isnan(e2).any(dim=1).all())
    m.sync_check()  # reported once
    m.embed(x, sync=False)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match=r"rc=-6"):
        m.embed(x)  # the next call reports the earlier async failure
    m.set_option(N.FR_OPT_STAGE_SPIN_LIMIT, 0)
    e3 = m.embed(x).cpu().numpy()
    assert np.array_equal(e3, good) and m.stage_reruns() == 1
    m.close()


def test_sync_embed_does_not_swallow_async_failure(gpu):
    """An FR_EMBED_ASYNC forward whose split-stage wait runs out, followed at once (no host sync) by a
    synchronous fr_embed: the failure belongs to the async forward and is reported as such (FR_ERR_STAGE
    from the synchronous call, which has not run), never taken by the synchronous call as its own and
    cleared by its re-run.  The next call then runs normally."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("iresnet100")
    x = torch.from_numpy(synthetic_crops(6, 112, seed=78)).cuda()
    m.set_option(N.FR_OPT_STAGE, 2)
    good = m.embed(x).cpu().numpy()
    m.set_option(N.FR_OPT_STAGE_SPIN_LIMIT, -1)
    e_async = m.embed(x, sync=False)
    with pytest.raises(RuntimeError, match=r"rc=-6"):
        m.embed(x)
    assert bool(torch.isnan(e_async).any(dim=1).all())
    assert m.stage_reruns() == 0  # the synchronous call did not re-run (it did not run at all)
    m.sync_check()  # reported once
    m.set_option(N.FR_OPT_STAGE_SPIN_LIMIT, 0)
    assert np.array_equal(m.embed(x).cpu().numpy(), good)
    m.close()


def test_two_handles_share_a_device(gpu):
    """Two handles on one device, forwards on two streams: their split-stage forwards are chained on
    the GPU (DevSerial), no wait runs out, and each result equals its single-handle result."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    a, b = FRModel.synthetic("iresnet100"), FRModel.synthetic("iresnet100")
    xa = torch.from_numpy(synthetic_crops(128, 112, seed=1)).cuda()
    xb = torch.from_numpy(synthetic_crops(128, 112, seed=2)).cuda()
    ra, rb = a.embed(xa).cpu().numpy(), b.embed(xb).cpu().numpy()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for _ in range(3):
        with torch.cuda.stream(sa):
            oa = a.embed(xa, sync=False)
        with torch.cuda.stream(sb):
            ob = b.embed(xb, sync=False)
        outs.append((oa, ob))
    torch.cuda.synchronize()
    for oa, ob in outs:
        assert np.array_equal(oa.cpu().numpy(), ra) and np.array_equal(ob.cpu().numpy(), rb)
    with torch.cuda.stream(sa):
        a.sync_check()
    with torch.cuda.stream(sb):
        b.sync_check()
    assert a.stage_timeouts() == 0 and b.stage_timeouts() == 0
    a.close()
    b.close()


@pytest.mark.parametrize("dtype,B", [("bf16", 5), ("f16", 3), ("bf16", 256)])
def test_stage_variants_bit_identical(gpu, dtype, B):
    """The 13-fragment layer3 stage kernel (default), the legacy 14-row layout (FR_OPT_STAGE_VARIANT 1), the
    one-wave-per-SIMD 13-fragment kernel (2) and the channel-split one (3) run the same K-steps and epilogue
    arithmetic: every layer3 intermediate and every embedding is
    bit-identical, at padded fragment counts and at the full bs = 256 grid."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("iresnet100", dtype=dtype)
    x = torch.from_numpy(synthetic_crops(B, 112, seed=60 + B))
    names = {"layer3.1.prelu", "layer3.1", "layer3.2.prelu", "layer3.15", "layer3.29"}
    m.set_option(N.FR_OPT_STAGE, 2)
    m.set_option(N.FR_OPT_KEEP_INTERMEDIATES, 1)
    out = {}
    for v in (0, 1, 2, 3):
        m.set_option(N.FR_OPT_STAGE_VARIANT, v)
        e = m.embed(x).cpu().numpy()
        out[v] = (e, _named(m, B, names))
    m.close()
    for v in (1, 2, 3):
        # (variant 1 has no layer3-stage tail: layer4.0.conv1 then runs per conv, in another f32 order, so only
        # the layer3 tensors are bit-identical there and the embeddings agree to rounding)
        if v == 1:
            cos = np.sum(out[0][0] * out[v][0], axis=1)
            assert (1 - cos).max() < 1e-4, (v, (1 - cos).max())
        else:
            assert np.array_equal(out[0][0], out[v][0]), v
        for n in names:
            assert torch.equal(out[0][1][n], out[v][1][n]), (v, n)
