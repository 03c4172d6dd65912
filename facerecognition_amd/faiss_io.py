"""Reader / writer of FAISS flat-index files (``faiss.write_index`` / ``faiss.read_index`` of an
IndexFlatIP / IndexFlatL2), so the reference's ``arcface_index.faiss`` galleries load into a
DeviceGallery without faiss (written by extract_embeddings.py:595-645, 871-872,
read by recognition_engine.py:142-146, 453).  faiss is not installed here; the layout below restates the
published format of faiss's impl/index_write.cpp for IndexFlat (faiss-cpu/-gpu >= 1.7.4, the
requirements-colab.txt:31 pin; the pre-1.7.3 layout is byte-identical), all little-endian:

    fourcc      4 B   "IxFI" (METRIC_INNER_PRODUCT), "IxF2" (METRIC_L2), "IxFl" (other metrics)
    d           int32 dimension
    ntotal      int64 number of vectors
    dummy       int64 1 << 20 (twice)
    is_trained  uint8
    metric_type int32 (0 = inner product, 1 = L2; a float metric_arg follows only when > 1)
    size        uint64 number of 4-byte words of the code array (= ntotal * d)
    codes       float32 [ntotal, d], row-major

No faiss file ships with the reference, so the format is parity unpinned: tests/test_faiss_io.py checks
it against a byte fixture assembled from the layout above."""
from __future__ import annotations

import struct
from typing import Tuple

import numpy as np

FOURCC = {0: b"IxFI", 1: b"IxF2"}
METRIC_INNER_PRODUCT, METRIC_L2 = 0, 1


def write_flat_index(path: str, rows: np.ndarray, metric: int = METRIC_INNER_PRODUCT) -> None:
    rows = np.ascontiguousarray(rows, dtype="<f4")
    n, d = rows.shape
    with open(path, "wb") as f:
        f.write(FOURCC.get(metric, b"IxFl"))
        f.write(struct.pack("<iqqqBi", d, n, 1 << 20, 1 << 20, 1, metric))
        f.write(struct.pack("<Q", n * d))
        f.write(rows.tobytes())


def read_flat_index(path: str) -> Tuple[np.ndarray, int]:
    """Returns (rows f32 [ntotal, d], metric_type).  Raises ValueError for anything that is not a flat
    index (IVF, HNSW, PQ, ... files: the reference only ever writes IndexFlatIP)."""
    with open(path, "rb") as f:
        buf = f.read()
    if len(buf) < 4 or buf[:4] not in (b"IxFI", b"IxF2", b"IxFl"):
        raise ValueError(f"{path}: not a FAISS flat index (fourcc {buf[:4]!r})")
    off = 4
    d, n, _, _, _trained, metric = struct.unpack_from("<iqqqBi", buf, off)
    off += struct.calcsize("<iqqqBi")
    if metric > 1:
        off += 4  # metric_arg (float)
    (size,) = struct.unpack_from("<Q", buf, off)
    off += 8
    if d <= 0 or n < 0 or size != n * d or len(buf) < off + 4 * size:
        raise ValueError(f"{path}: inconsistent FAISS flat index header (d={d}, ntotal={n}, size={size})")
    rows = np.frombuffer(buf, dtype="<f4", count=size, offset=off).reshape(n, d).astype(np.float32)
    return rows, metric
