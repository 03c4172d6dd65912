"""Face detector host logic on the CPU: facerecognition_amd.face_detector.detect_face
(the product's thresholding / NMS / box arithmetic, numpy float32) driven by the CPU oracle's P/R/O-nets
and area resampler (oracle/mtcnn.py, test infrastructure) must reproduce oracle.mtcnn.detect_face -- the
restatement of facenet-pytorch 2.5.x's detect_face -- exactly: same boxes, probabilities and landmarks,
in the same order.  MTCNN is parity unpinned (facenet-pytorch and its weights are absent; synthetic
weights, synth_mtcnn_state).  The device nets are checked against the same oracle in
tests/test_gpu_face_detector.py."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from facerecognition_amd import face_detector as FD
from oracle import mtcnn as OM


def synthetic_scene(seed, H=150, W=190, coarse=4):
    """Smooth random RGB u8 image (bicubic-upsampled noise)."""
    rng = np.random.default_rng(seed)
    a = torch.tensor(rng.standard_normal((H // coarse + 2, W // coarse + 2, 3)))
    a = F.interpolate(a.permute(2, 0, 1)[None], size=(H, W), mode="bicubic", align_corners=False)[0].permute(1, 2, 0)
    a = a.numpy()
    return ((a - a.min()) / (a.max() - a.min()) * 255).clip(0, 255).astype(np.uint8)


def oracle_callables(nets):
    """The oracle's nets behind detect_face's callable contract (NHWC in, concatenated heads out)."""
    pn, rn, on = nets

    def resample(imgs, regions, oh, ow):
        x = torch.as_tensor(np.asarray(imgs)).permute(0, 3, 1, 2).float()
        out = [OM.imresample(x[r[0]:r[0] + 1, :, r[1]:r[1] + r[3], r[2]:r[2] + r[4]], (oh, ow)) for r in regions]
        return ((torch.cat(out, 0) - 127.5) * 0.0078125).permute(0, 2, 3, 1)

    def nchw(x):
        return x.permute(0, 3, 1, 2).contiguous()

    def pnet(x):
        reg, prob = pn(nchw(x))
        return torch.cat([prob, reg], 1).permute(0, 2, 3, 1)

    def rnet(x):
        reg, prob = rn(nchw(x))
        return torch.cat([prob, reg], 1)

    def onet(x):
        reg, lm, prob = on(nchw(x))
        return torch.cat([prob, reg, lm], 1)

    return resample, pnet, rnet, onet


class _Contig(torch.nn.Module):
    """A net fed contiguous NCHW: the oracle's pyramid levels are channels-last views, and the CPU conv's
    rounding depends on the memory format; both pipelines see the same layout through this wrapper."""

    def __init__(self, m):
        super().__init__()
        self.m = m

    def forward(self, x):
        return self.m(x.contiguous())


@pytest.fixture(scope="module")
def nets():
    return tuple(_Contig(m) for m in OM.build_nets(FD.synth_mtcnn_state(7)))


@pytest.mark.parametrize("seed,coarse", [(0, 4), (1, 3), (2, 6), (3, 2)])
def test_host_logic_matches_oracle_detect_face(nets, seed, coarse):
    img = synthetic_scene(seed, coarse=coarse)
    with torch.no_grad():
        rb, rp = OM.detect_face(img[None], *nets)
        gb, gp = FD.detect_face(img[None], *oracle_callables(nets))
    assert len(rb[0]) > 10, "the synthetic weights should leave detections through all three stages"
    assert gb[0].shape == rb[0].shape
    assert np.array_equal(gb[0], rb[0])
    assert np.array_equal(gp[0], rp[0])


def test_batch_of_two_images(nets):
    imgs = np.stack([synthetic_scene(5), synthetic_scene(6)])
    with torch.no_grad():
        rb, rp = OM.detect_face(imgs, *nets)
        gb, gp = FD.detect_face(imgs, *oracle_callables(nets))
    for b in range(2):
        assert np.array_equal(gb[b], rb[b]) and np.array_equal(gp[b], rp[b])


def test_nms_modes_against_oracle():
    rng = np.random.default_rng(0)
    xy = rng.uniform(0, 100, (300, 2)).astype(np.float32)
    wh = rng.uniform(5, 40, (300, 2)).astype(np.float32)
    boxes = np.concatenate([xy, xy + wh], 1)
    scores = rng.uniform(0, 1, 300).astype(np.float32)
    scores[10] = scores[20]  # a tie
    for t in (0.3, 0.5, 0.7):
        assert np.array_equal(FD.nms(boxes, scores, t, "iou"), OM.nms_iou(boxes, scores, t))
        assert np.array_equal(FD.nms(boxes, scores, t, "min"), OM.nms_numpy(boxes, scores, t, "Min"))


def test_nms_grid_windows_against_oracle():
    """PNet-like windows (a dense 12-px grid at stride 2, scaled boxes of several pyramid levels, near-equal
    scores) and degenerate boxes (zero / negative extent: numpy's 0 / 0 drops them regardless of distance):
    the grid-bucketed fr_nms_host keeps exactly the numpy greedy pass's boxes, in its order."""
    rng = np.random.default_rng(4)
    parts = []
    for s in (1.0, 0.7, 0.49):
        yy, xx = np.mgrid[0:30, 0:40].astype(np.float32)
        q1 = np.floor((2 * np.stack([xx.ravel(), yy.ravel()], 1) + 1) / s)
        q2 = np.floor((2 * np.stack([xx.ravel(), yy.ravel()], 1) + 12) / s)
        parts.append(np.concatenate([q1, q2], 1))
    boxes = np.concatenate(parts + [np.array([[5, 5, 5, 9], [50, 50, 50, 50], [80, 10, 70, 20], [7, 7, 7, 7]], np.float32)])
    boxes = boxes.astype(np.float32)
    scores = np.round(rng.uniform(0.6, 1.0, len(boxes)), 2).astype(np.float32)  # many exact ties
    for t in (0.5, 0.7):
        assert np.array_equal(FD.nms(boxes, scores, t, "iou"), OM.nms_iou(boxes, scores, t))
        assert np.array_equal(FD.nms(boxes, scores, t, "min"), OM.nms_numpy(boxes, scores, t, "Min"))


def test_batched_nms_many_frames_against_oracle():
    """batched_nms over B = 16 frames (the coordinate-offset trick spreads them along a diagonal, so a dense class
    grid would grow as B^2 cells: ADVICE r05): the same kept set as the oracle's per-image pass, in bounded time."""
    import time
    rng = np.random.default_rng(9)
    B, per = 16, 2000
    xy = rng.uniform(0, 1900, (B * per, 2)).astype(np.float32)
    wh = rng.choice([12.0, 24.0, 48.0, 300.0], (B * per, 1)).astype(np.float32)
    boxes = np.concatenate([xy, xy + wh], 1)
    scores = np.round(rng.uniform(0.6, 1.0, B * per), 3).astype(np.float32)
    inds = np.repeat(np.arange(B), per)
    t0 = time.perf_counter()
    got = FD.batched_nms(boxes, scores, inds, 0.5, "iou")
    dt = time.perf_counter() - t0
    off = inds.astype(np.float32) * (boxes.max() + np.float32(1))
    ref = OM.nms_iou((boxes + off[:, None]).astype(np.float32), scores, 0.5)
    assert np.array_equal(got, ref)
    assert dt < 2.0, f"batched_nms over {B} frames took {dt:.2f} s"


def test_pyramid_and_pool_shapes():
    assert FD.pyramid_scales(150, 190) == OM.pyramid_scales(150, 190)
    for n in range(2, 60):
        for k, s in ((2, 2), (3, 2)):
            if n >= k:
                assert FD.pool_ceil_out(n, k, s) == F.max_pool2d(torch.zeros(1, 1, n, n), k, s, ceil_mode=True).shape[-1]


def test_face_detector_selection_rules(nets):
    """_detect_mtcnn's confidence / minimum-size / largest-face selection on the oracle's MTCNN.detect."""
    img = synthetic_scene(0)
    det = OM.face_detector_detect(np.ascontiguousarray(img[..., ::-1]), nets)
    assert det is not None and det["confidence"] >= 0.9
    x1, y1, x2, y2 = det["bbox"]
    assert min(x2 - x1, y2 - y1) >= 19 and set(det["landmarks"]) == set(FD.LANDMARK_NAMES)
