"""Crop preparation restatements on CPU (oracle/preprocess.py, facerecognition_amd/align.py).

The Pillow resize restatement is pinned to PIL itself (installed here and on the GPU box); the cv2 warp
and the skimage similarity estimate are parity unpinned (neither library is installed) and are checked
by their defining properties instead."""
import os

import numpy as np
import pytest
from PIL import Image

from facerecognition_amd.align import ARCFACE_TEMPLATE, similarity_transform
from oracle.preprocess import cv2_warp_affine, pillow_resize

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _pil(img, w, h):
    return np.asarray(Image.fromarray(img).resize((w, h), Image.BILINEAR))


@pytest.mark.parametrize("shape,out", [((900, 900), (112, 112)), ((50, 50), (112, 112)), ((113, 113), (112, 112)),
                                       ((200, 150), (112, 112)), ((97, 230), (160, 160)), ((112, 300), (112, 112)),
                                       ((300, 112), (112, 112))])
def test_pillow_resize_restatement_matches_pil(shape, out):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    img = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    if shape == (900, 900):
        with np.load(os.path.join(GOLD, "anh1_u8.npz"), allow_pickle=False) as z:
            img = z["u8"]
    assert np.array_equal(pillow_resize(img, out[1], out[0]), _pil(img, out[1], out[0]))


def test_similarity_transform_recovers_known_similarity():
    rng = np.random.default_rng(3)
    for _ in range(5):
        s, th = rng.uniform(0.3, 3.0), rng.uniform(-np.pi, np.pi)
        R = s * np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
        t = rng.uniform(-100, 100, 2)
        src = rng.uniform(0, 300, (5, 2))
        dst = src @ R.T + t
        T = similarity_transform(src, dst)
        assert np.allclose(T[:2, :2], R, atol=1e-9) and np.allclose(T[:2, 2], t, atol=1e-7)
    # reflection-free even for mirrored input, and rank-deficient (all-equal points) gives NaN like skimage
    assert np.isnan(similarity_transform(np.ones((5, 2)), ARCFACE_TEMPLATE)).all()


def test_cv2_warp_restatement_properties():
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (60, 70, 3), dtype=np.uint8)
    # identity and integer translations copy pixels exactly; the uncovered border is 0
    assert np.array_equal(cv2_warp_affine(img, np.array([[1.0, 0, 0], [0, 1.0, 0]]), 70, 60), img)
    sh = cv2_warp_affine(img, np.array([[1.0, 0, 5], [0, 1.0, -3]]), 70, 60)
    assert np.array_equal(sh[0:57, 5:], img[3:60, 0:65]) and not sh[:, :5].any() and not sh[57:].any()
    # a half-pixel shift averages neighbours with the round-half-up fixed point of OpenCV
    half = cv2_warp_affine(img, np.array([[1.0, 0, -0.5], [0, 1.0, 0]]), 69, 60)
    ref = (img[:, :69].astype(int) * 16384 * 32 // 32 + img[:, 1:70].astype(int) * 16384 + (1 << 14)) >> 15
    assert np.array_equal(half, np.clip(ref, 0, 255).astype(np.uint8))
