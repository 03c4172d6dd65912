"""FAISS flat-index files without faiss (facerecognition_amd/faiss_io.py; the reference writes and reads
them at extract_embeddings.py:642 / recognition_engine.py:145).  faiss is not installed and no .faiss
file ships with the reference, so the layout is checked against a byte fixture assembled field by field
from faiss's published index_write.cpp layout (parity unpinned)."""
import struct

import numpy as np
import pytest

from facerecognition_amd import faiss_io as F


def _fixture_bytes(rows, fourcc=b"IxFI", metric=0):
    n, d = rows.shape
    b = bytearray(fourcc)
    b += struct.pack("<i", d)                 # d
    b += struct.pack("<q", n)                 # ntotal
    b += struct.pack("<q", 1 << 20) * 2       # two dummy idx_t
    b += struct.pack("<B", 1)                 # is_trained
    b += struct.pack("<i", metric)            # metric_type
    b += struct.pack("<Q", n * d)             # code words
    b += rows.astype("<f4").tobytes()
    return bytes(b)


def test_write_matches_byte_fixture(tmp_path):
    rows = np.arange(12, dtype=np.float32).reshape(3, 4) / 7
    p = str(tmp_path / "a.faiss")
    F.write_flat_index(p, rows)
    assert open(p, "rb").read() == _fixture_bytes(rows)


def test_read_fixture_and_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    rows = rng.standard_normal((5, 512)).astype(np.float32)
    p = tmp_path / "b.faiss"
    p.write_bytes(_fixture_bytes(rows))
    got, metric = F.read_flat_index(str(p))
    assert metric == 0 and np.array_equal(got, rows)
    p2 = str(tmp_path / "c.faiss")
    F.write_flat_index(p2, rows, metric=F.METRIC_L2)
    got, metric = F.read_flat_index(p2)
    assert metric == 1 and np.array_equal(got, rows) and open(p2, "rb").read()[:4] == b"IxF2"
    empty = str(tmp_path / "e.faiss")
    F.write_flat_index(empty, np.zeros((0, 8), np.float32))
    got, _ = F.read_flat_index(empty)
    assert got.shape == (0, 8)


def test_rejects_other_index_types(tmp_path):
    p = tmp_path / "ivf.faiss"
    p.write_bytes(b"IwFl" + b"\0" * 64)
    with pytest.raises(ValueError):
        F.read_flat_index(str(p))
    rows = np.ones((2, 4), np.float32)
    bad = bytearray(_fixture_bytes(rows))
    bad[-9] ^= 0xFF  # truncate the code array's claimed size against the payload
    p.write_bytes(bytes(bad[:-8]))
    with pytest.raises(ValueError):
        F.read_flat_index(str(p))


def test_facenet_web_match_oracle_semantics():
    """oracle.match.facenet_web_match restates web_app.py:537-559: rows renormalized, distance output,
    stable order on ties, threshold."""
    from oracle.match import facenet_web_match
    e = np.array([1.0, 0.0, 0.0, 0.0], np.float32)
    db = {"a": np.array([2.0, 0, 0, 0], np.float32), "b": np.array([0.0, 1, 0, 0], np.float32),
          "c": np.array([3.0, 0, 0, 0], np.float32)}
    name, score, dist, top = facenet_web_match(e, db, 0.5)
    assert name == "a" and [t[0] for t in top] == ["a", "c", "b"]
    assert abs(score - 1.0) < 1e-6 and dist < 1e-6 and abs(top[2][2] - np.sqrt(2)) < 1e-6
    assert facenet_web_match(np.array([0, 0, 1.0, 0], np.float32), db, 0.5)[0] == "Unknown"
