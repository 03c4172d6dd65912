"""Host-side logic of the reference-compatible API, without a GPU: result conventions, thresholds,
naming quirks, db file loading, the build-job state machine, and argument errors.  The compute
behind these calls (fr_embed / fr_match_topk) is covered by the -m gpu tests."""
import os
import pickle

import numpy as np
import pytest

from facerecognition_amd import database_builder as DB
from facerecognition_amd import extract_embeddings as EE
from facerecognition_amd import recognition_engine as RE
from oracle import match as OMT

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "arcface_r50_golden.npz")


def test_cosine_similarity_matches_reference_golden():
    with np.load(GOLD, allow_pickle=False) as z:
        a, cases = z["emb_single"][0], z["cos_cases"]
    rng = np.random.default_rng(0)
    g = rng.standard_normal(512).astype(np.float32)
    g /= np.linalg.norm(g)
    for b in (g, 3 * g, np.zeros(512, np.float32)):
        assert RE.cosine_similarity(a, b) == OMT.cosine_similarity(a, b)
    with np.load(GOLD, allow_pickle=False) as z:
        from facerecognition_amd.synthetic import planted_gallery
        G = planted_gallery(z["emb_batch"], int(z["gallery_rows"]), seed=int(z["gallery_seed"]))
    got = [RE.cosine_similarity(a, G[7]), RE.cosine_similarity(a, G[7] * 3.0),
           RE.cosine_similarity(a, np.zeros(512, np.float32))]
    assert np.allclose(got, cases, atol=1e-6)


def test_db_file_round_trip_reference_format(tmp_path):
    db = {"alice": np.arange(4, dtype=np.float32), "bob": np.ones(4, np.float32)}
    p = str(tmp_path / "db.npy")
    np.save(p, db)  # exactly how the reference writes it (extract_embeddings.py:826, save_db :428)
    got = RE.load_npy_object(p)
    assert list(got) == ["alice", "bob"]
    assert all(np.array_equal(got[k], db[k]) for k in db)
    arr = np.arange(6, dtype=np.float32)
    np.save(str(tmp_path / "a.npy"), arr)
    assert np.array_equal(RE.load_npy_object(str(tmp_path / "a.npy")), arr)


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned > /dev/null",))


def test_db_loader_refuses_code(tmp_path):
    from numpy.lib import format as npf
    p = tmp_path / "evil.npy"
    with open(p, "wb") as f:
        npf.write_array_header_1_0(f, {"descr": "|O", "fortran_order": False, "shape": ()})
        pickle.dump(_Evil(), f, protocol=3)
    with pytest.raises(pickle.UnpicklingError):
        RE.load_npy_object(str(p))


def test_tracked_db_counts_mutations():
    d = RE._TrackedDB({"a": 1})
    v = d.version
    d["b"] = 2
    d.update(c=3)
    del d["a"]
    d.pop("b")
    assert d.version == v + 4 and dict(d) == {"c": 3}


def test_engine_without_model_or_db_follows_reference_conventions():
    eng = RE.RecognitionEngine(model_path=None, use_face_detection=False)
    assert eng.recognize_with_db(np.ones(512, np.float32)) == ("No database", 0.0, [])
    assert eng.recognize_with_faiss(np.ones(512, np.float32)) == ("No FAISS index", 0.0, [])
    r = eng.recognize("does-not-exist.jpg")
    assert r["status"] == "error" and r["identity"] == "Unknown" and r["embedding"] is None
    assert r["message"] == "Cannot extract embedding (no face or invalid image)"
    assert eng.extract_embedding("x.jpg") is None
    assert eng.get_db_identities() == []
    assert eng.add_to_db("x", []) is False


def test_face_detection_request_falls_back_like_reference(capsys):
    eng = RE.RecognitionEngine(model_path=None, use_face_detection=True)
    assert eng.use_face_detection is False and eng.face_detector is None
    assert "Face Detector" in capsys.readouterr().out


def test_result_threshold_and_names():
    eng = RE.RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.5)
    names = ["a", "b", "c"]
    assert eng._result_db(np.array([0.9, 0.4, 0.1]), np.array([2, 0, 1]), names) == \
        ("c", 0.9, [("c", 0.9), ("a", 0.4), ("b", 0.1)])
    name, score, top = eng._result_db(np.array([0.3, 0.2], np.float32), np.array([1, 0]), names)
    assert name == "Unknown" and abs(score - 0.3) < 1e-7 and top[0][0] == "b"
    # FAISS path: id_to_label maps name -> label, so integer lookups miss (reference quirk kept)
    eng.id_to_label = {"alice": 0, "bob": 1}
    assert eng._result_faiss(np.array([0.8, 0.7]), np.array([1, 0]))[0] == "ID_1"
    assert eng._result_faiss(np.array([-np.inf]), np.array([-1])) == ("Unknown", 0.0, [])


def mixed_norm_case():
    """A db and probes that exercise every cosine_similarity branch (recognition_engine.py:41-63),
    including a near-tie that flips if a unit-ish probe (|p| = 1.0009) is rescaled against a raw
    unit-ish row or left unscaled against a normalized non-unit row."""
    D = 8
    e = np.eye(D, dtype=np.float32)
    c_a = 0.8
    c_b = c_a * 1.0009 * (1 - 5e-4)  # reference: A (0.80072) beats B (0.80032); wrong rule: B (0.80104) wins
    A = c_a * e[0] + np.sqrt(1 - c_a ** 2) * e[1]
    B = 2.0 * (c_b * e[0] + np.sqrt(1 - c_b ** 2) * e[2])
    rng = np.random.default_rng(4)
    db = {"A": A, "B": B, "zero": np.zeros(D, np.float32), "near": 1.0005 * e[3], "big": 3.0 * e[4]}
    for j in range(12):
        v = np.zeros(D, np.float32)
        v[5:] = rng.standard_normal(D - 5)
        v[0] = 0.3 * rng.standard_normal()
        db[f"r{j}"] = v / np.linalg.norm(v) * (1.0 if j % 3 else 2.5)
    probes = [1.0009 * e[0], e[0], 2.0 * e[0], np.zeros(D, np.float32), 1.0005 * e[3] + 0.01 * e[4],
              rng.standard_normal(D).astype(np.float32)]
    return {k: np.asarray(v, np.float32) for k, v in db.items()}, [np.asarray(p, np.float32) for p in probes]


class _NumpyGallery:
    """Stand-in for DeviceGallery on the CPU (host-logic test only): fr_gallery_set's row preparation
    (rows off unit norm by >= 1e-3 are normalized, zero rows stay zero) + exact top-k."""

    def __init__(self, rows, dim=512, device=0):
        import torch
        r = np.asarray(rows, np.float32).reshape(-1, dim).copy()
        n = np.linalg.norm(r, axis=1)
        fix = (np.abs(n - 1) >= 1e-3) & (n > 0)
        r[fix] /= n[fix, None]
        self.rows, self.device = r, torch.device("cpu")

    @property
    def ntotal(self):
        return len(self.rows)

    def _prep(self, rows):
        r = np.asarray(rows, np.float32).reshape(-1, self.rows.shape[1]).copy()
        n = np.linalg.norm(r, axis=1)
        fix = (np.abs(n - 1) >= 1e-3) & (n > 0)
        r[fix] /= n[fix, None]
        return r

    def add(self, rows):  # fr_gallery_write append
        self.rows = np.concatenate([self.rows, self._prep(rows)], 0)

    def update(self, row0, rows):  # fr_gallery_write in place
        r = self._prep(rows)
        self.rows[row0:row0 + len(r)] = r

    def search_device(self, P, k):
        import torch
        s, i = OMT.topk_dot(P.numpy(), self.rows, k)
        return torch.from_numpy(s), torch.from_numpy(i.astype(np.int32))


def test_recognize_with_db_mixed_norm_semantics(monkeypatch):
    from facerecognition_amd import gallery
    monkeypatch.setattr(gallery, "DeviceGallery", _NumpyGallery)
    db, probes = mixed_norm_case()
    eng = RE.RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.0)
    eng.db = db
    for p in probes:
        name, score, top = eng.recognize_with_db(p)
        rname, rscore, rtop = OMT.recognize_with_db(p, db, 0.0)
        assert name == rname and [t[0] for t in top] == [t[0] for t in rtop]
        assert np.allclose([t[1] for t in top], [t[1] for t in rtop], atol=1e-6)
    assert eng.recognize_with_db(probes[0])[0] == "A"  # the near-tie resolves as the reference does


def test_db_edits_apply_in_place_and_match_a_rebuild(monkeypatch):
    """add_to_db-style edits (new names, re-assigned names in the same norm class) are applied to the
    device copy in place (no rebuild); a class change or a deletion rebuilds; every state answers like
    the reference's recognize_with_db over the same dict."""
    from facerecognition_amd import gallery
    monkeypatch.setattr(gallery, "DeviceGallery", _NumpyGallery)
    db, probes = mixed_norm_case()
    eng = RE.RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.0)
    eng.db = dict(db)
    rng = np.random.default_rng(9)

    def check():
        for p in probes + [rng.standard_normal(8).astype(np.float32)]:
            name, _, top = eng.recognize_with_db(p)
            rname, _, rtop = OMT.recognize_with_db(p, dict(eng.db), 0.0)
            assert name == rname and [t[0] for t in top] == [t[0] for t in rtop]
            assert np.allclose([t[1] for t in top], [t[1] for t in rtop], atol=1e-6)

    check()
    parts0 = eng._g[1]
    v = rng.standard_normal(8).astype(np.float32)
    eng.db["new_unit"] = v / np.linalg.norm(v)      # append to 'on'
    eng.db["new_off"] = 2.0 * v                     # append to 'off'
    eng.db["A"] = np.roll(db["A"], 1)               # same class, in place
    check()
    assert eng._g[1] is parts0, "journaled edits must not rebuild the device copy"
    eng.db["big"] = db["big"] / 3.0                 # 'off' -> 'on': rebuild
    check()
    assert eng._g[1] is not parts0
    parts1 = eng._g[1]
    del eng.db["B"]                                 # deletion: rebuild
    check()
    assert eng._g[1] is not parts1


def test_shared_db_journal_per_engine(monkeypatch):
    """Two engines holding ONE db: each replays the journal entries past its own synced version, so an
    engine that syncs first does not empty the journal the other still needs."""
    from facerecognition_amd import gallery
    monkeypatch.setattr(gallery, "DeviceGallery", _NumpyGallery)
    db, probes = mixed_norm_case()
    e1 = RE.RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.0)
    e2 = RE.RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.0)
    e1.db = dict(db)
    e2.db = e1.db
    rng = np.random.default_rng(5)

    def check(eng):
        for p in probes:
            name, _, top = eng.recognize_with_db(p)
            rname, _, rtop = OMT.recognize_with_db(p, dict(eng.db), 0.0)
            assert name == rname and [t[0] for t in top] == [t[0] for t in rtop]

    check(e1)
    check(e2)
    p1, p2 = e1._g[1], e2._g[1]
    for i in range(3):
        v = rng.standard_normal(8).astype(np.float32)
        e1.db[f"n{i}"] = v / np.linalg.norm(v)
        check(e1)  # e1 syncs after every edit; e2 only at the end, replaying all three
    e1.db["A"] = probes[0] / np.linalg.norm(probes[0])  # a probe-like row: must win for e2 too
    check(e1)
    check(e2)
    assert e1._g[1] is p1 and e2._g[1] is p2, "journaled edits must not rebuild either device copy"
    assert e2.recognize_with_db(probes[0])[0] == "A"
    del e1.db["B"]  # restarts the journal: both rebuild
    check(e1)
    check(e2)
    assert e2._g[1] is not p2


def test_extract_batch_empty_and_bad_paths():
    emb, paths = EE.extract_embeddings_batch([], model=None, transform=EE.get_transform())
    assert emb.size == 0 and paths == []
    emb, paths = EE.extract_embeddings_batch(["/nonexistent/a.jpg"], model=None, transform=EE.get_transform())
    assert emb.size == 0 and paths == []
    assert EE.extract_embedding_single("/nonexistent/a.jpg", None, EE.get_transform()) is None


def test_device_strings():
    assert EE._device_index("cuda") == 0 and EE._device_index("cuda:3") == 3 and EE._device_index(2) == 2
    with pytest.raises(ValueError):
        EE._device_index("cpu")


def test_compute_prototypes_matches_oracle(tmp_path):
    rng = np.random.default_rng(3)
    E = rng.standard_normal((40, 16)).astype(np.float32)
    L = rng.integers(0, 5, 40)
    L[:5] = np.arange(5)
    got = EE.compute_prototypes(E, L, str(tmp_path / "p.npy"))
    assert np.array_equal(got, OMT.compute_prototypes(E, L))
    assert np.array_equal(np.load(tmp_path / "p.npy"), got)


def test_transform_resizes_with_pil_bilinear():
    from PIL import Image
    rng = np.random.default_rng(1)
    img = Image.fromarray(rng.integers(0, 256, (200, 180, 3), dtype=np.uint8))
    t = EE.get_transform(112)
    x = t(img).numpy()
    ref = np.asarray(img.resize((112, 112), Image.BILINEAR), dtype=np.float32).transpose(2, 0, 1) / 255
    assert x.shape == (3, 112, 112) and np.allclose(x, (ref - 0.5) / 0.5, atol=1e-6)
    assert EE.get_facenet_transform().size == 160


# ---------------------------------------------------------------------------------------- builder
def _run(builder, job_id, model_type, config):
    builder.create_job(job_id, model_type, config)
    builder.start_build(job_id).join(30)
    return builder.get_job(job_id)


def test_build_job_completes_and_records_outputs():
    calls = []
    b = DB.DatabaseBuilder(build_fn=lambda **kw: calls.append(kw))
    job = _run(b, "j1", "arcface", {"model_path": "m.pth", "data_dir": "d"})
    assert job.status == "completed" and job.progress == 100.0 and job.error is None
    assert job.output_files == {"ArcFace Database": "data/arcface_embeddings_db.npy"}
    assert calls[0]["model_type"] == "arcface" and calls[0]["root_folder"] == "d" and calls[0]["device"] == "cuda"
    d = job.to_dict()
    assert set(d) == {"job_id", "model_type", "status", "progress", "message", "logs", "output_files", "error",
                      "elapsed_time"}
    job = _run(b, "j2", "facenet", {"data_dir": "d", "output_path": "x.npy"})
    assert job.output_files == {"FaceNet Database": "x.npy"} and calls[1]["model_type"] == "facenet"


def test_build_job_failures():
    def boom(**kw):
        raise RuntimeError("disk full")
    b = DB.DatabaseBuilder(build_fn=boom)
    job = _run(b, "f", "arcface", {})
    assert job.status == "failed" and job.error == "disk full" and any("Traceback" in l for l in job.logs)
    assert _run(b, "l", "lbph", {}).status == "failed"
    bad = _run(b, "x", "sift", {})
    assert bad.status == "failed" and "không hợp lệ" in bad.error
    with pytest.raises(ValueError):
        b.start_build("missing")
    assert DB.get_builder() is DB.get_builder()


def test_build_job_logs_capped():
    j = DB.BuildJob("a", "arcface", {})
    for n in range(80):
        j.add_log(str(n))
    assert len(j.to_dict()["logs"]) == 50 and j.to_dict()["elapsed_time"] is None
    j.update_progress(150)
    assert j.progress == 100.0


def test_transform_size_must_match_model():
    """the device resize targets the transform's image_size, and a transform whose size is not
    the model's input side is an error (the reference would feed the model a wrong-size crop)."""
    import facerecognition_amd.extract_embeddings as EE

    class _M:
        arch, input_size = "iresnet100", 112
    EE._check_transform(_M(), EE.get_transform(112))
    with pytest.raises(ValueError):
        EE._check_transform(_M(), EE.get_transform(160))
    with pytest.raises(TypeError):
        EE._check_transform(_M(), object())
    assert EE.extract_embedding_single(np.zeros((112, 112, 3), np.uint8), _M(), EE.get_transform(160)) is None
