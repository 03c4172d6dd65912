"""numpy restatements of the reference's match / gallery code (TEST INFRASTRUCTURE ONLY)."""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np


def cosine_similarity(a: np.ndarray, b: np.ndarray) -> float:
    """inference/recognition_engine.py:41-63."""
    a = a.astype(np.float32).flatten()
    b = b.astype(np.float32).flatten()
    na, nb = np.linalg.norm(a), np.linalg.norm(b)
    if na == 0 or nb == 0:
        return 0.0
    if abs(na - 1.0) < 1e-3 and abs(nb - 1.0) < 1e-3:
        return float(np.dot(a, b))
    return float(np.dot(a, b) / (na * nb))


def recognize_with_db(embedding: np.ndarray, db: Dict[str, np.ndarray], threshold: float
                      ) -> Tuple[str, float, List[Tuple[str, float]]]:
    """inference/recognition_engine.py:267-289 (stable sort: ties keep insertion order)."""
    if db is None:
        return "No database", 0.0, []
    scores = [(name, cosine_similarity(embedding, vec)) for name, vec in db.items()]
    scores.sort(key=lambda x: x[1], reverse=True)
    best_name, best_score = scores[0]
    if best_score < threshold:
        return "Unknown", best_score, scores[:5]
    return best_name, best_score, scores[:5]


def topk_dot(P: np.ndarray, G: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Notebook batched match (evaluate_arcface_kaggle.ipynb cells 15-16: np.dot + argmax /
    argsort) with the order made total: score desc, index asc (np.argmax's first-max rule).
    Rows beyond N are padded with (-inf, -1) like FAISS."""
    S = np.dot(P.astype(np.float32), G.astype(np.float32).T)
    B, Nn = S.shape
    kk = min(k, Nn)
    idx = np.lexsort((np.broadcast_to(np.arange(Nn), S.shape), -S), axis=1)[:, :kk]
    sc = np.take_along_axis(S, idx, 1)
    if kk < k:
        sc = np.concatenate([sc, np.full((B, k - kk), -np.inf, np.float32)], 1)
        idx = np.concatenate([idx, np.full((B, k - kk), -1)], 1)
    return sc.astype(np.float32), idx.astype(np.int64)


def argmax_top1(P: np.ndarray, G: np.ndarray) -> np.ndarray:
    """evaluate_arcface_kaggle.ipynb cell 15: np.argmax(np.dot(emb, prototypes.T), axis=1)."""
    return np.argmax(np.dot(P, G.T), axis=1)


def faiss_flat_ip_search(G: np.ndarray, P: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """IndexFlatIP over rows normalized by build_faiss_index (extract_embeddings.py:625-627),
    probe normalized by recognize_with_faiss (recognition_engine.py:300-301)."""
    G = G.astype(np.float32)
    G = G / (np.linalg.norm(G, axis=1, keepdims=True) + 1e-8)
    P = P.astype(np.float32).reshape(-1, G.shape[1])
    P = P / (np.linalg.norm(P, axis=1, keepdims=True) + 1e-8)
    return topk_dot(P, G, k)


def folder_mean(embs: np.ndarray) -> np.ndarray:
    """extract_embedding_for_folder tail (extract_embeddings.py:755-760) / add_to_db
    (recognition_engine.py:411-413) / compute_prototypes (:585-588)."""
    m = np.mean(np.stack(embs, axis=0), axis=0)
    return m / (np.linalg.norm(m) + 1e-8)


def compute_prototypes(embeddings: np.ndarray, labels: np.ndarray) -> np.ndarray:
    """inference/extract_embeddings.py:555-592."""
    unique = np.unique(labels)
    protos = np.zeros((len(unique), embeddings.shape[1]), dtype=np.float32)
    for lab in unique:
        p = embeddings[labels == lab].mean(axis=0)
        protos[lab] = p / (np.linalg.norm(p) + 1e-8)
    return protos


def merge_topk(cand_s: np.ndarray, cand_i: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Merge of per-shard candidate lists [P, n_lists, k] → [P, k] with the same total order as
    topk_dot (score desc, global index asc; (-inf, -1) padding sorts last).  No reference
    counterpart: this is the exchange step of the multi-GPU design."""
    P = cand_s.shape[0]
    s = cand_s.reshape(P, -1).astype(np.float32)
    i = cand_i.reshape(P, -1).astype(np.int64)
    key_i = np.where(i < 0, np.iinfo(np.int64).max, i)
    order = np.lexsort((key_i, -s), axis=1)[:, :k]
    return np.take_along_axis(s, order, 1), np.take_along_axis(i, order, 1)


def facenet_web_match(embedding: np.ndarray, db: Dict[str, np.ndarray], threshold: float):
    """web_app.py:537-559 (the FaceNet recognition route): probe / (|e| + 1e-8); every db row renormalized
    by (|row| + 1e-8); score = dot, distance = |e - row|; stable sort by score desc; best < threshold ->
    "Unknown".  Returns (identity, confidence, distance, top_k[:5] as (name, score, distance))."""
    e = np.asarray(embedding, dtype=np.float32).flatten()
    e = e / (np.linalg.norm(e) + 1e-8)
    top_k = []
    for name, db_emb in db.items():
        r = np.asarray(db_emb, dtype=np.float32).flatten()
        r = r / (np.linalg.norm(r) + 1e-8)
        top_k.append((name, float(np.dot(e, r)), float(np.linalg.norm(e - r))))
    top_k.sort(key=lambda x: x[1], reverse=True)
    best_name, best_score, best_distance = top_k[0]
    if best_score < threshold:
        best_name = "Unknown"
    return best_name, best_score, best_distance, top_k[:5]
