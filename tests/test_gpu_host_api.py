"""The reference-compatible host API end to end on the GPU, checked against the reference's own
outputs (tests/golden/arcface_r50_golden.npz, produced by importing the reference's
ArcFaceModel / extract_embedding_single / RecognitionEngine.recognize_with_db; tools/gen_golden.py).

Tolerances: embeddings within 1e-3 cosine distance of the reference's (north star);
match scores of given embeddings within 1e-5 (f32 dot products, different summation order);
indices / names identical."""
import os

import numpy as np
import pytest

from facerecognition_amd import _native as N

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "arcface_r50_golden.npz")
COS_TOL = 1e-3


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLD, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def r50(gold, gpu):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.weights import synth_state_dict
    sd = synth_state_dict("resnet50_arcface", seed=int(gold["seed"]), num_classes=int(gold["num_classes"]))
    return FRModel("resnet50_arcface", sd, max_batch=64)


@pytest.fixture(scope="module")
def names_db(gold):
    from facerecognition_amd.synthetic import planted_gallery
    G = planted_gallery(gold["emb_batch"], int(gold["gallery_rows"]), seed=int(gold["gallery_seed"]))
    names = [f"id_{i:04d}" for i in range(len(G))]
    return names, {n: G[i] for i, n in enumerate(names)}


def _cos_dist(a, b):
    a = a / np.linalg.norm(a, axis=-1, keepdims=True)
    b = b / np.linalg.norm(b, axis=-1, keepdims=True)
    return 1 - (a * b).sum(-1)


def test_extract_embedding_single_vs_reference(gold, r50):
    from PIL import Image
    from facerecognition_amd.extract_embeddings import extract_embedding_single, get_transform
    t = get_transform()
    got = np.stack([extract_embedding_single(Image.fromarray(p), r50, t) for p in gold["probes"]])
    assert got.dtype == np.float32 and got.shape == (8, 512)
    assert _cos_dist(got, gold["emb_single"]).max() <= COS_TOL


def test_natural_image_tensor_vs_reference(gold, r50):
    """uploads/anh1.jpg after the reference transform (f32 NCHW input path of fr_embed)."""
    import torch
    e = r50.embed(torch.from_numpy(gold["natural_tensor"])[None]).cpu().numpy()[0]
    assert _cos_dist(e, gold["natural_emb"]) <= COS_TOL


def test_raw_forward_vs_reference(gold, r50):
    import torch
    raw = r50(torch.from_numpy(gold["probes"])).cpu().numpy()  # ArcFaceModel(x, labels=None): unnormalized
    assert _cos_dist(raw, gold["emb_raw"]).max() <= COS_TOL
    n_ref, n = np.linalg.norm(gold["emb_raw"], axis=1), np.linalg.norm(raw, axis=1)
    assert np.allclose(n, n_ref, rtol=5e-3)


def test_recognize_with_db_vs_reference(gold, names_db):
    from facerecognition_amd.recognition_engine import RecognitionEngine
    names, db = names_db
    eng = RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.5)
    eng.db = db
    for p in range(8):
        name, score, top5 = eng.recognize_with_db(gold["emb_single"][p])
        assert name == str(gold["best_name"][p])
        assert [names.index(t[0]) for t in top5] == list(gold["top5_idx"][p])
        assert np.allclose([t[1] for t in top5], gold["top5_scores"][p], atol=1e-5)
    eng.db = {"dup_a": db["id_0003"], "dup_b": db["id_0003"].copy(), "other": db["id_0005"]}
    name, _, top = eng.recognize_with_db(gold["emb_single"][3])
    assert name == str(gold["tie_name"]) and [t[0] for t in top] == list(gold["tie_top"])
    eng.db = db
    eng.set_threshold(0.999)
    name, score, _ = eng.recognize_with_db(gold["emb_single"][0])
    assert name == "Unknown" and abs(score - float(gold["unknown_score"])) < 1e-5


def test_recognize_batch_end_to_end(gold, r50, names_db):
    from PIL import Image
    from facerecognition_amd.recognition_engine import RecognitionEngine
    _, db = names_db
    # a caller-supplied model keeps its own setting unless batch_invariant is given (no silent re-tune of
    # a shared handle)
    RecognitionEngine(model_path=None, use_face_detection=False, model=r50)
    assert r50.get_option(N.FR_OPT_BATCH_INVARIANT) == 0
    eng = RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.5, model=r50, batch_invariant=True)
    eng.db = db
    imgs = [Image.fromarray(p) for p in gold["probes"]] + ["/nonexistent.jpg"]
    res = eng.recognize_batch(imgs)
    assert [r["identity"] for r in res[:8]] == [str(n) for n in gold["best_name"]]
    assert res[8]["status"] == "error" and res[8]["embedding"] is None
    single = eng.recognize(imgs[2])
    # batch_invariant=True: recognize_batch is bit for bit a loop over recognize, as the reference's recognize_batch
    # is (recognition_engine.py:383-389)
    assert r50.get_option(N.FR_OPT_BATCH_INVARIANT) == 1
    assert np.array_equal(single["embedding"], res[2]["embedding"])
    assert single["identity"] == res[2]["identity"] and single["confidence"] == res[2]["confidence"]
    assert _cos_dist(single["embedding"], gold["emb_single"][2]) <= COS_TOL
    assert _cos_dist(res[2]["embedding"], gold["emb_single"][2]) <= COS_TOL
    # in-place db edit is picked up by the device copy
    eng.db["zz_probe2"] = res[2]["embedding"]
    assert eng.recognize(imgs[2])["identity"] == "zz_probe2"
    r50.set_option(N.FR_OPT_BATCH_INVARIANT, 0)  # the shared fixture goes back to the throughput default


def test_folder_db_build_and_faiss_path(gold, r50, tmp_path):
    from PIL import Image
    import torch
    from facerecognition_amd import extract_embeddings as EE
    from facerecognition_amd.recognition_engine import RecognitionEngine, create_engine_from_embeddings_dir
    from oracle.match import faiss_flat_ip_search, folder_mean
    for person, idx in (("p0", [0, 1, 2]), ("p1", [3, 4]), ("p2", [5, 6, 7])):
        os.makedirs(tmp_path / "celeb" / person)
        for i in idx:
            Image.fromarray(gold["probes"][i]).save(tmp_path / "celeb" / person / f"{i}.png")
    t = EE.get_transform()
    e = EE.extract_embedding_for_folder(str(tmp_path / "celeb" / "p1"), r50, t)
    assert _cos_dist(e, folder_mean(gold["emb_single"][[3, 4]])) <= COS_TOL
    # checkpoint in the reference's schema -> build_db -> RecognitionEngine(db_path)
    from facerecognition_amd.weights import synth_state_dict
    sd = synth_state_dict("resnet50_arcface", seed=int(gold["seed"]), num_classes=int(gold["num_classes"]))
    ck = str(tmp_path / "arcface_best.pth")
    torch.save({"model_state_dict": {k: torch.as_tensor(v) for k, v in sd.items()},
                "config": {"num_classes": 100, "model": {"embedding_size": 512}}, "epoch": 3}, ck)
    dbp = str(tmp_path / "db.npy")
    EE.build_db(ck, str(tmp_path / "celeb"), dbp, "cuda", use_face_detection=False)
    eng = RecognitionEngine(model_path=ck, db_path=dbp, use_face_detection=False, threshold=0.3)
    assert sorted(eng.get_db_identities()) == ["p0", "p1", "p2"]
    assert eng.recognize(Image.fromarray(gold["probes"][4]))["identity"] == "p1"
    # FAISS-style index over the same identities
    protos = np.stack([eng.db[k] for k in ("p0", "p1", "p2")])
    os.makedirs(tmp_path / "emb")
    EE.build_faiss_index(protos, str(tmp_path / "emb" / "arcface_index.faiss"))  # FAISS file format
    eng2 = create_engine_from_embeddings_dir(ck, str(tmp_path / "emb"), threshold=0.3)
    name, score, res = eng2.recognize_with_faiss(gold["emb_single"][6], k=3)
    s_ref, i_ref = faiss_flat_ip_search(protos, gold["emb_single"][6], 3)
    assert [r[0] for r in res] == [f"ID_{i}" for i in i_ref[0]]
    assert np.allclose([r[1] for r in res], s_ref[0], atol=1e-5)


def test_extract_embeddings_batch_vs_reference(gold, r50, tmp_path):
    """extract_embeddings_batch (extract_embeddings.py:392-443) on image files, batch_size 3 so the
    chunks are ragged; a bad path in the middle is skipped and left out of valid_paths."""
    from PIL import Image
    from facerecognition_amd import extract_embeddings as EE
    paths = []
    for i, p in enumerate(gold["probes"]):
        f = str(tmp_path / f"{i}.png")
        Image.fromarray(p).save(f)
        paths.append(f)
    paths.insert(4, str(tmp_path / "missing.png"))
    emb, valid = EE.extract_embeddings_batch(paths, r50, EE.get_transform(), batch_size=3)
    assert valid == [p for p in paths if "missing" not in p]
    assert emb.dtype == np.float32 and emb.shape == (8, 512)
    assert _cos_dist(emb, gold["emb_batch"]).max() <= COS_TOL


def test_natural_image_u8_path_vs_reference(gold, r50):
    """uploads/anh1.jpg decoded (tests/golden/anh1_u8.npz) -> host PIL resize -> fused u8 path."""
    from PIL import Image
    from facerecognition_amd.extract_embeddings import extract_embedding_single, get_transform
    with np.load(os.path.join(os.path.dirname(GOLD), "anh1_u8.npz"), allow_pickle=False) as z:
        u8 = z["u8"]
    e = extract_embedding_single(Image.fromarray(u8), r50, get_transform())
    assert _cos_dist(e, gold["natural_emb"]) <= COS_TOL


def test_recognize_with_db_mixed_norm_on_device():
    """cosine_similarity's per-pair rule (both norms within 1e-3 of 1 -> dot, else dot / |a||b|)
    through the device galleries, including the near-tie that the old probe-only rescaling flipped."""
    from facerecognition_amd.recognition_engine import RecognitionEngine
    from oracle.match import recognize_with_db
    from test_host_api import mixed_norm_case
    db, probes = mixed_norm_case()
    eng = RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.0)
    eng.db = db
    for p in probes:
        name, score, top = eng.recognize_with_db(p)
        rname, rscore, rtop = recognize_with_db(p, db, 0.0)
        assert name == rname and [t[0] for t in top] == [t[0] for t in rtop]
        assert np.allclose([t[1] for t in top], [t[1] for t in rtop], atol=1e-6)
    assert eng.recognize_with_db(probes[0])[0] == "A"


def test_database_builder_end_to_end(gold, tmp_path):
    """DatabaseBuilder.create_job / start_build (database_builder.py:184-234) -> build_db with every
    identity's crops in shared fr_embed batches + one fr_segment_mean_normalize launch -> the reference's
    dict .npy; rows equal the folder means of the reference's own embeddings (golden emb_single)."""
    from PIL import Image
    import torch
    from facerecognition_amd import database_builder as DB
    from facerecognition_amd.recognition_engine import load_npy_object
    from facerecognition_amd.weights import synth_state_dict
    from oracle.match import folder_mean
    groups = {"p0": [0, 1, 2], "p1": [3, 4], "p2": [5, 6, 7], "empty": []}
    for person, idx in groups.items():
        os.makedirs(tmp_path / "celeb" / person)
        for i in idx:
            Image.fromarray(gold["probes"][i]).save(tmp_path / "celeb" / person / f"{i}.png")
    (tmp_path / "celeb" / "p1" / "notes.txt").write_text("not an image")
    sd = synth_state_dict("resnet50_arcface", seed=int(gold["seed"]), num_classes=int(gold["num_classes"]))
    ck = str(tmp_path / "arcface_best.pth")
    torch.save({"model_state_dict": {k: torch.as_tensor(v) for k, v in sd.items()},
                "config": {"num_classes": 100, "model": {"embedding_size": 512}}}, ck)
    out = str(tmp_path / "db.npy")
    b = DB.DatabaseBuilder()
    b.create_job("j", "arcface", {"model_path": ck, "data_dir": str(tmp_path / "celeb"), "output_path": out,
                                  "use_face_detection": False})
    b.start_build("j").join(300)
    job = b.get_job("j")
    assert job.status == "completed", job.logs
    db = load_npy_object(out)
    assert sorted(db) == ["p0", "p1", "p2"]  # the identity with no image is skipped, as the reference
    for person, idx in groups.items():
        if idx:
            assert _cos_dist(db[person], folder_mean(gold["emb_single"][idx])) <= COS_TOL


def test_segment_means_many_identities(r50):
    """segment_means over 300 identities of 1-3 crops (spans two 256-image fr_embed batches): each row
    equals the host mean / renorm of that identity's fr_embed outputs."""
    import torch
    from facerecognition_amd.extract_embeddings import segment_means
    from facerecognition_amd.synthetic import synthetic_crops
    from oracle.match import folder_mean
    u8 = synthetic_crops(600, 112, seed=40)
    sizes = [1 + (g % 3) for g in range(300)]
    groups, o = [], 0
    for n in sizes:
        groups.append(list(u8[o:o + n]))
        o += n
    groups.insert(7, [])
    rows = segment_means(r50, groups)
    assert rows[7] is None
    # the same 256-image batches as segment_means, so the per-image embeddings are bit-identical
    E = np.concatenate([r50.embed(torch.from_numpy(u8[a:min(a + 256, o)])).cpu().numpy() for a in range(0, o, 256)])
    o = 0
    for g, n in enumerate(sizes):
        row = rows[g if g < 7 else g + 1]
        assert np.allclose(row, folder_mean(E[o:o + n]), atol=2e-6)
        o += n


def test_facenet_matcher_vs_web_route():
    """FaceNetMatcher (device) vs the web route's loop (web_app.py:537-559): renormalized rows (some
    far from unit norm), names / order, scores, distances, threshold."""
    from facerecognition_amd.recognition_engine import FaceNetMatcher
    from oracle.match import facenet_web_match
    rng = np.random.default_rng(8)
    db = {f"id{j}": rng.standard_normal(512).astype(np.float32) * (1.0 if j % 4 else 3.0) for j in range(300)}
    probes = [db["id5"] * 0.5 + 0.1 * rng.standard_normal(512).astype(np.float32),
              rng.standard_normal(512).astype(np.float32), 2.0 * db["id12"]]
    m = FaceNetMatcher(db, threshold=0.3)
    for p, got in zip(probes, m.match_batch(np.stack(probes))):
        name, score, dist, top = facenet_web_match(p, db, 0.3)
        assert got["identity"] == name and [t[0] for t in got["top_k"]] == [t[0] for t in top]
        assert abs(got["confidence"] - score) < 1e-5 and abs(got["distance"] - dist) < 1e-5
        assert np.allclose([t[2] for t in got["top_k"]], [t[2] for t in top], atol=1e-5)


def test_db_edits_in_place_on_device():
    """The journaled add_to_db edits through the real device galleries (fr_gallery_write) answer like the
    reference's recognize_with_db over the same dict, before and after a rebuild."""
    from facerecognition_amd.recognition_engine import RecognitionEngine
    from oracle.match import recognize_with_db
    from test_host_api import mixed_norm_case
    db, probes = mixed_norm_case()
    eng = RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.0)
    eng.db = dict(db)
    rng = np.random.default_rng(10)

    def check():
        for p in probes:
            name, _, top = eng.recognize_with_db(p)
            rname, _, rtop = recognize_with_db(p, dict(eng.db), 0.0)
            assert name == rname and [t[0] for t in top] == [t[0] for t in rtop]
            assert np.allclose([t[1] for t in top], [t[1] for t in rtop], atol=1e-6)

    check()
    parts0 = eng._g[1]
    for j in range(40):  # many single-row appends (capacity growth) + in-place updates
        v = rng.standard_normal(8).astype(np.float32)
        eng.db[f"n{j}"] = v / np.linalg.norm(v) if j % 2 else 3.0 * v
        if j % 7 == 0:
            eng.db["A"] = np.roll(db["A"], j % 3)
        check()
    assert eng._g[1] is parts0
