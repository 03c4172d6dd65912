"""Device MTCNN (facerecognition_amd/face_detector.py + mtcnn.hip) against the CPU restatement of
facenet-pytorch's MTCNN (oracle/mtcnn.py; parity unpinned: facenet-pytorch and its weights are absent, the
weights are synth_mtcnn_state).  The area resampler is bit-exact; the f32 nets agree to float rounding
(tolerances below); end to end, boxes, probabilities and landmarks agree, and so does the reference's
FaceDetector selection and the engine's detect -> align -> embed path."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from facerecognition_amd import face_detector as FD
from oracle import mtcnn as OM
from tests.test_face_detector import synthetic_scene

pytestmark = pytest.mark.gpu

NET_RTOL = 1e-4


@pytest.fixture(scope="module")
def mt(gpu):
    state = FD.synth_mtcnn_state(7)
    return FD.DeviceMTCNN(state, device=0), OM.build_nets(state)


def test_area_resample_bit_exact(mt):
    dev, _ = mt
    rng = np.random.default_rng(1)
    imgs = rng.integers(0, 256, (2, 97, 131, 3), dtype=np.uint8)
    regions = np.array([[0, 0, 0, 97, 131], [1, 0, 0, 97, 131], [1, 10, 7, 40, 33], [0, 50, 60, 47, 71],
                        [1, 3, 100, 5, 9]], np.int32)
    x = torch.as_tensor(imgs).permute(0, 3, 1, 2).float()
    for oh, ow in ((24, 24), (48, 48), (69, 93), (13, 7)):
        got = dev.resample(torch.as_tensor(imgs).cuda(), regions, oh, ow).cpu()
        ref = torch.cat([F.interpolate(x[r[0]:r[0] + 1, :, r[1]:r[1] + r[3], r[2]:r[2] + r[4]], size=(oh, ow),
                                       mode="area") for r in regions])
        ref = ((ref - 127.5) * 0.0078125).permute(0, 2, 3, 1)
        assert torch.equal(got, ref), (oh, ow)


def _rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def test_nets_match_oracle(mt):
    dev, (pn, rn, on) = mt
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        x = torch.rand(2, 57, 73, 3, generator=g) * 2 - 1
        out = dev.pnet(x.cuda()).cpu()
        reg, prob = pn(x.permute(0, 3, 1, 2))
        assert _rel(out[..., :2], prob.permute(0, 2, 3, 1)) < NET_RTOL
        assert _rel(out[..., 2:], reg.permute(0, 2, 3, 1)) < NET_RTOL
        x = torch.rand(37, 24, 24, 3, generator=g) * 2 - 1
        out = dev.rnet(x.cuda()).cpu()
        reg, prob = rn(x.permute(0, 3, 1, 2).contiguous())
        assert _rel(out[:, :2], prob) < NET_RTOL and _rel(out[:, 2:], reg) < NET_RTOL
        x = torch.rand(29, 48, 48, 3, generator=g) * 2 - 1
        out = dev.onet(x.cuda()).cpu()
        reg, lm, prob = on(x.permute(0, 3, 1, 2).contiguous())
        assert _rel(out[:, :2], prob) < NET_RTOL and _rel(out[:, 2:6], reg) < NET_RTOL
        assert _rel(out[:, 6:], lm) < NET_RTOL


@pytest.mark.parametrize("seed,coarse", [(0, 4), (1, 3), (2, 6), (3, 2)])
def test_detect_face_matches_oracle(mt, seed, coarse):
    """Same detections as the fp32 CPU restatement: the f32 device nets move probabilities by ~1e-6, so a
    threshold or NMS decision can only differ for a candidate within that of a threshold (reported)."""
    dev, nets = mt
    img = synthetic_scene(seed, coarse=coarse)
    with torch.no_grad():
        rb, rp = OM.detect_face(img[None], *nets)
    gb, gp = dev.detect_face(img[None])
    rb, rp, gb, gp = rb[0], rp[0], gb[0], gp[0]
    print(f"scene {seed}: {len(gb)} device / {len(rb)} oracle detections")
    assert len(rb) > 10 and len(gb) == len(rb)
    assert np.allclose(gb[:, 4], rb[:, 4], atol=1e-5)
    assert np.allclose(gb[:, :4], rb[:, :4], atol=2e-3)
    assert np.allclose(gp, rp, atol=2e-3)


def test_face_detector_and_engine_alignment(mt, gpu):
    """FaceDetector.detect (the reference's _detect_mtcnn selection) equals the oracle's; the engine's
    detect_and_align warps that face to ARCFACE_TEMPLATE on the device and embeds the aligned crop."""
    from facerecognition_amd.align import align_faces
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.recognition_engine import RecognitionEngine
    dev, nets = mt
    fdet = FD.FaceDetector(mtcnn_state=FD.synth_mtcnn_state(7))
    for seed in range(4):
        bgr = np.ascontiguousarray(synthetic_scene(seed)[..., ::-1])
        got, ref = fdet.detect(bgr), OM.face_detector_detect(bgr, nets)
        assert (got is None) == (ref is None)
        if got is not None:
            assert got["bbox"] == ref["bbox"] and abs(got["confidence"] - ref["confidence"]) < 1e-5
            for k in FD.LANDMARK_NAMES:
                assert np.allclose(got["landmarks"][k], ref["landmarks"][k], atol=2e-3)
    model = FRModel.synthetic("resnet50_arcface")
    eng = RecognitionEngine(model_path=None, model=model, use_face_detection=True, face_detector=fdet)
    assert eng.use_face_detection and eng.face_detector is fdet
    rgb = synthetic_scene(0)
    det = fdet.detect_rgb(rgb)
    aligned, ok = align_faces(torch.as_tensor(rgb)[None].cuda(), [det["landmarks"]])
    assert ok[0]
    pil = eng.detect_and_align(np.ascontiguousarray(rgb[..., ::-1]))
    assert np.array_equal(np.asarray(pil), aligned[0].cpu().numpy())
    e1 = eng.extract_embedding(np.ascontiguousarray(rgb[..., ::-1]))
    e2 = model.embed(aligned.cpu()).cpu().numpy()[0]
    assert np.allclose(e1, e2, atol=1e-6)


def test_calibrated_weights_1080p_matches_oracle(gpu):
    """tools/mtcnn_bench.py's headline case: the calibrated synthetic weights (trained-detector box volumes) on
    its smooth 1080p frame -- the same detections as the CPU restatement."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from mtcnn_bench import frame
    state = FD.synth_mtcnn_state(7, calibrated=True)
    dev, nets = FD.DeviceMTCNN(state, device=0), OM.build_nets(state)
    img = frame()
    with torch.no_grad():
        rb, rp = OM.detect_face(img[None], *nets)
    FD.STATS = {}
    try:
        gb, gp = dev.detect_face(img[None])
        counts = dict(FD.STATS)
    finally:
        FD.STATS = None
    rb, rp, gb, gp = rb[0], rp[0], gb[0], gp[0]
    print(f"1080p calibrated: {len(gb)} device / {len(rb)} oracle detections; P-net passes {counts.get('pnet_pass_n')}, "
          f"R-net inputs {counts.get('rnet_ms_n')}, O-net inputs {counts.get('onet_ms_n')}")
    assert len(rb) > 0 and len(gb) == len(rb)
    assert np.allclose(gb[:, 4], rb[:, 4], atol=1e-5)
    assert np.allclose(gb[:, :4], rb[:, :4], atol=2e-3)
    assert np.allclose(gp, rp, atol=2e-3)
