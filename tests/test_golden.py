"""The oracle pinned to the reference's own outputs (CPU only).

tests/golden/arcface_r50_golden.npz was produced by tools/gen_golden.py, which imported the
reference's models/arcface/arcface_model.py, inference/extract_embeddings.py and
inference/recognition_engine.py unchanged (shims only for the absent torchvision / cv2 modules)
and ran them on synthetic weights + synthetic crops.  Here the oracle restatement (oracle/) must
reproduce those outputs; the GPU path is then checked against the oracle (tests/test_gpu_*.py).
"""
import os

import numpy as np
import pytest
import torch

from facerecognition_amd.synthetic import planted_gallery, synthetic_crops
from facerecognition_amd.weights import synth_state_dict
from oracle import match as OMT
from oracle import models as OM

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "arcface_r50_golden.npz")


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLD, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def oracle_model(gold):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    sd = synth_state_dict("resnet50_arcface", seed=int(gold["seed"]), num_classes=int(gold["num_classes"]))
    return OM.build_model("resnet50_arcface", sd, num_classes=int(gold["num_classes"]))


def test_probe_generator_is_stable(gold):
    assert np.array_equal(synthetic_crops(8, 112, seed=0), gold["probes"])


def test_oracle_embeddings_match_reference(gold, oracle_model):
    emb = OM.embed(oracle_model, "resnet50_arcface", gold["probes"])
    assert np.abs(emb - gold["emb_batch"]).max() < 1e-5
    assert np.abs(emb - gold["emb_single"]).max() < 1e-5
    with torch.no_grad():
        raw = oracle_model(OM.preprocess_u8_nhwc(gold["probes"]), labels=None).numpy()
    assert np.abs(raw - gold["emb_raw"]).max() < 1e-4 * np.abs(gold["emb_raw"]).max()


def test_oracle_natural_image_embedding(gold, oracle_model):
    """uploads/anh1.jpg (900x900) after the reference transform (PIL bilinear resize to 112)."""
    with torch.no_grad():
        e = oracle_model(torch.from_numpy(gold["natural_tensor"])[None], labels=None)
        e = torch.nn.functional.normalize(e, dim=1).numpy()[0]
    assert np.abs(e - gold["natural_emb"]).max() < 1e-5


def test_host_transform_matches_reference_on_natural_image(gold):
    """The 900x900 -> 112x112 PIL bilinear Resize + ToTensor + Normalize of the host transform equals
    the reference transform's output (golden natural_tensor) on uploads/anh1.jpg, decoded pixels in
    tests/golden/anh1_u8.npz (tools/gen_natural_fixture.py)."""
    from facerecognition_amd.extract_embeddings import get_transform
    from PIL import Image
    with np.load(os.path.join(os.path.dirname(GOLD), "anh1_u8.npz"), allow_pickle=False) as z:
        u8 = z["u8"]
    assert u8.shape == (900, 900, 3)
    t = get_transform()
    x = t(Image.fromarray(u8)).numpy()
    assert x.shape == (3, 112, 112)
    assert np.abs(x - gold["natural_tensor"]).max() <= 1e-6
    # and the identity-resize path on the synthetic crops
    x = t(Image.fromarray(gold["probes"][0])).numpy()
    assert np.array_equal(x, OM.preprocess_u8_nhwc(gold["probes"][:1]).numpy()[0])


def _gallery(gold):
    G = planted_gallery(gold["emb_batch"], int(gold["gallery_rows"]), seed=int(gold["gallery_seed"]))
    assert abs(G.astype(np.float64).sum() - float(gold["gallery_sum"])) < 1e-9
    return G


def test_recognize_with_db_restatement(gold):
    G = _gallery(gold)
    names = [f"id_{i:04d}" for i in range(len(G))]
    db = {n: G[i] for i, n in enumerate(names)}
    for p in range(len(gold["emb_single"])):
        name, score, top5 = OMT.recognize_with_db(gold["emb_single"][p], db, 0.5)
        assert name == str(gold["best_name"][p])
        assert [names.index(t[0]) for t in top5] == list(gold["top5_idx"][p])
        assert np.allclose([t[1] for t in top5], gold["top5_scores"][p], atol=1e-6)
    name, score, _ = OMT.recognize_with_db(gold["emb_single"][0], db, 0.999)
    assert name == str(gold["unknown_name"]) == "Unknown"
    assert abs(score - float(gold["unknown_score"])) < 1e-6


def test_tie_order_and_cosine_branches(gold):
    G = _gallery(gold)
    db = {"dup_a": G[3], "dup_b": G[3].copy(), "other": G[5]}
    name, _, top = OMT.recognize_with_db(gold["emb_single"][3], db, 0.5)
    assert name == str(gold["tie_name"]) and [t[0] for t in top] == list(gold["tie_top"])
    a = gold["emb_single"][0]
    got = [OMT.cosine_similarity(a, G[7]), OMT.cosine_similarity(a, G[7] * 3.0),
           OMT.cosine_similarity(a, np.zeros(512, np.float32))]
    assert np.allclose(got, gold["cos_cases"], atol=1e-6)


def test_batched_match_restatement(gold):
    G = _gallery(gold)
    assert np.array_equal(OMT.argmax_top1(gold["emb_batch"], G), gold["argmax"])
    _, idx = OMT.topk_dot(gold["emb_batch"], G, 5)
    assert np.array_equal(idx[:, 0], gold["argmax"])
    assert np.array_equal(idx, gold["top5_idx"])
