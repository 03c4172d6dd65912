"""Drop-in for the reference's ``inference/recognition_engine.py`` (RecognitionEngine, cosine_similarity,
create_engine_from_embeddings_dir) with embedding and gallery matching on the MI355X.

Reference → here:
  cosine_similarity :41-63            unchanged host function (a10)
  RecognitionEngine.__init__ :75-140  same arguments; dict db (.npy) and/or index + prototypes + mapping
  extract_embedding :244-265          fr_embed via extract_embedding_single (a7)
  recognize_with_db :267-289          fr_match_topk against the device copy of the db (dict order =
                                       row order; (score desc, index asc) = the stable sort), top-5,
                                       cosine_similarity's both-norms-unit rule per pair (_db_gallery),
                                       ``best < threshold`` → "Unknown"; no db → ("No database", 0.0, [])
  recognize_with_faiss :291-326       probe / (‖p‖+1e-8), exact inner-product top-k on the device
                                       index; names ``id_to_label.get(idx, f"ID_{idx}")`` (reference quirk kept)
  recognize :328-381                  same result dict / status / message
  recognize_batch :383-389            batched: all images in one fr_embed + one fr_match_topk (§8f row 1)
  add_to_db / save_db / get_db_identities / set_threshold :391-435, :165-167
  FaceNetMatcher                      the FaceNet web route's matcher (web_app.py:537-559): renormalized
                                       rows, score + L2 distance, threshold
  detect_and_align / align_face :169-242  device MTCNN (face_detector.FaceDetector) +
                                       the device 5-point warp to ARCFACE_TEMPLATE (align.align_faces); the
                                       crop fallback when a face has no landmarks.  Without MTCNN weights
                                       the detector is unavailable and the engine runs on the raw image:
                                       the reference's own fallback without facenet-pytorch (:122-124).

The device gallery is rebuilt lazily whenever the db changes (``engine.db = {...}``, ``add_to_db``, or
item assignment on ``engine.db``).  Scores are f32 inner products computed on the GPU; they agree with
the reference's numpy ``cosine_similarity`` to ~1e-6 (accumulation order), and ranks are identical
except between rows whose scores differ by less than that.
"""
from __future__ import annotations

import io
import os
import pickle
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _native as N
from . import weights as Wt
from .extract_embeddings import (_device_index, _embed_u8, _load_u8, extract_embedding_single,
                                 get_transform, load_arcface_model, read_index, segment_means)

MAX_K = 4096  # fr_match_topk limit (k > 16: exact score rows + a device radix select)


def cosine_similarity(a: np.ndarray, b: np.ndarray) -> float:
    a = a.flatten().astype(np.float32)
    b = b.flatten().astype(np.float32)
    na, nb = np.linalg.norm(a), np.linalg.norm(b)
    if na == 0 or nb == 0:
        return 0.0
    if abs(na - 1.0) < 1e-3 and abs(nb - 1.0) < 1e-3:
        return float(np.dot(a, b))
    return float(np.dot(a, b) / (na * nb))


# ---------------------------------------------------------------------------------------- db files
class _NumpyOnlyUnpickler(pickle.Unpickler):
    """The reference stores its db / label mapping as ``np.save(path, dict)`` (a pickled 0-d object
    array).  Load those with an unpickler that can only rebuild numpy arrays, dtypes and plain
    containers — never arbitrary callables."""
    ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
               ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
               ("numpy", "ndarray"), ("numpy", "dtype"), ("builtins", "dict"), ("builtins", "list"),
               ("builtins", "tuple"), ("builtins", "str"), ("builtins", "int"), ("builtins", "float"),
               ("collections", "OrderedDict"), ("_codecs", "encode")}

    def find_class(self, module, name):
        if (module, name) in self.ALLOWED or (module.startswith("numpy") and name.startswith("dtype")):
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a db file")


def load_npy_object(path: str):
    """np.load(path, allow_pickle=True).item() restricted to numpy/builtin types."""
    from numpy.lib import format as npf
    with open(path, "rb") as f:
        version = npf.read_magic(f)
        read_header = npf.read_array_header_1_0 if version == (1, 0) else npf.read_array_header_2_0
        _shape, _fortran, dtype = read_header(f)
        if dtype != object:
            return np.load(path, allow_pickle=False)
        arr = _NumpyOnlyUnpickler(io.BytesIO(f.read())).load()
    return arr.item() if isinstance(arr, np.ndarray) and arr.shape == () else arr


class _Grow:
    """A numpy vector with amortised O(1) append (capacity doubling); `view` is the live prefix."""

    def __init__(self, a):
        a = np.asarray(a)
        self._buf = np.empty(max(16, 2 * len(a)), dtype=a.dtype)
        self._buf[:len(a)] = a
        self._n = len(a)

    def append(self, x):
        if self._n == len(self._buf):
            self._buf = np.concatenate([self._buf, np.empty_like(self._buf)])
        self._buf[self._n] = x
        self._n += 1

    @property
    def view(self):
        return self._buf[:self._n]


class _TrackedDB(dict):
    """dict that counts mutations so the device copy knows when to refresh, and journals plain item
    assignments (the add_to_db / db[name] = emb pattern) so a device copy can apply them in place
    instead of rebuilding; any other mutation (del, pop, clear, ...) restarts the journal, so copies
    synced before it rebuild.  The journal is shared by every consumer (several engines may hold one
    db): entry i is the key assigned at version journal_base + i + 1, and each consumer replays the
    entries past the version it synced (journal_since)."""
    version = 0
    journal_base = 0
    JOURNAL_MAX = 1 << 16  # past this, the older half is dropped (consumers that far behind rebuild)

    @property
    def journal(self):
        if "_journal" not in self.__dict__:
            self._journal = []
        return self._journal

    def journal_since(self, version):
        """Keys assigned after `version` in order, or None when the journal does not reach back to it."""
        if version < self.journal_base or version > self.version:
            return None
        return self.journal[version - self.journal_base:]

    def _bump(self, key=None):
        self.version += 1
        if key is None:
            self.journal.clear()
            self.journal_base = self.version
            return
        self.journal.append(key)
        if len(self.journal) > self.JOURNAL_MAX:
            drop = len(self.journal) // 2
            del self.journal[:drop]
            self.journal_base += drop

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        self._bump(k)

    def __delitem__(self, k):
        super().__delitem__(k)
        self._bump()

    def update(self, *a, **k):
        for key, v in dict(*a, **k).items():
            self[key] = v

    def pop(self, *a):
        r = super().pop(*a)
        self._bump()
        return r

    def popitem(self):
        r = super().popitem()
        self._bump()
        return r

    def clear(self):
        super().clear()
        self._bump()

    def setdefault(self, k, v=None):
        if k not in self:
            self[k] = v
        return self[k]


class RecognitionEngine:
    def __init__(self, model_path: str = "models/checkpoints/arcface/arcface_best.pth", db_path: str = None,
                 faiss_index_path: str = None, prototypes_path: str = None, label_mapping_path: str = None,
                 device: str = None, threshold: float = 0.5, use_face_detection: bool = True, model=None,
                 face_detector=None, mtcnn_weights: str = None, batch_invariant: Optional[bool] = None):
        """batch_invariant: True runs the model with FR_OPT_BATCH_INVARIANT, so ``recognize_batch`` returns bit for
        bit what a loop over ``recognize`` returns, as the reference's does (recognition_engine.py:383-389); False
        lets the model pick the fastest kernels per batch size (embeddings then differ by ~1e-4 cosine between
        batch sizes).  None (default): True for a model the engine loads itself; a caller-supplied ``model=`` keeps
        its own setting (the option re-tunes the handle, which other users of a shared model would feel).  An
        explicit True/False is applied to a supplied model too.  fp8 models cannot be batch-invariant (their e4m3
        convs scale by a per-batch amax): they stay in the default mode, with a warning when True was asked."""
        self.device = device or "cuda"
        self.threshold = threshold
        self.use_face_detection = use_face_detection
        self.model, self.model_info = None, None
        owned = False
        if model is not None:  # an already-built FRModel (tests, services sharing one model)
            self.model = model
        elif model_path and os.path.exists(model_path):
            self.model, self.model_info = load_arcface_model(model_path, self.device)
            owned = True
        inv = owned if batch_invariant is None else bool(batch_invariant)
        if self.model is not None and (inv or batch_invariant is not None):
            if inv and getattr(self.model, "dtype", None) == "fp8":
                if batch_invariant:
                    print("batch_invariant: not available for fp8 models; the model keeps per-batch kernels")
            else:
                self.model.set_option(N.FR_OPT_BATCH_INVARIANT, 1 if inv else 0)
        self.transform = get_transform(Wt.INPUT_SIZE[self.model.arch] if self.model is not None else 112)
        self.face_detector = face_detector
        if self.use_face_detection and self.face_detector is None:
            try:
                from .face_detector import FaceDetector
                self.face_detector = FaceDetector(backend="mtcnn", device=self.device, confidence_threshold=0.9,
                                                  select_largest=True, weights_dir=mtcnn_weights)
                print("Face detector initialized (MTCNN)")
            except Exception as e:  # reference :122-124
                print(f"Khong the khoi tao Face Detector: {e}")
                self.use_face_detection = False
        self._db = None
        self._g = None          # (key, DeviceGallery, names)
        self.faiss_index = None
        self.prototypes = None
        self.label_to_id = None
        self.id_to_label = None
        if db_path and os.path.exists(db_path):
            self.db = load_npy_object(db_path)
            print(f"Loaded database: {len(self.db)} identities")
        if faiss_index_path and (os.path.exists(faiss_index_path) or os.path.exists(faiss_index_path + ".npz")):
            self._load_faiss(faiss_index_path, prototypes_path, label_mapping_path)

    # ------------------------------------------------------------------ state
    @property
    def db(self):
        return self._db

    @db.setter
    def db(self, value):
        self._db = None if value is None else (value if isinstance(value, _TrackedDB) else _TrackedDB(value))
        self._g = None

    def _load_faiss(self, index_path: str, prototypes_path: str = None, mapping_path: str = None):
        try:
            self.faiss_index = read_index(index_path)
            print(f"Loaded index: {self.faiss_index.ntotal} vectors")
        except Exception as e:
            print(f"Loi load FAISS: {e}")
            return
        if prototypes_path and os.path.exists(prototypes_path):
            self.prototypes = np.load(prototypes_path)
            print(f"Loaded prototypes: {self.prototypes.shape}")
        if mapping_path and os.path.exists(mapping_path):
            mapping = load_npy_object(mapping_path)
            self.label_to_id = mapping.get("label_to_id", {})
            self.id_to_label = mapping.get("id_to_label", {})
            print(f"Loaded label mapping: {len(self.label_to_id)} classes")

    def set_threshold(self, threshold: float):
        self.threshold = threshold
        print(f"Threshold set to: {threshold}")

    def align_face(self, image: np.ndarray, landmarks: Dict) -> Optional[np.ndarray]:
        """5-point similarity warp of a u8 [H, W, 3] image to ARCFACE_TEMPLATE (112 x 112, border 0) on the
        device (reference :169-204: skimage SimilarityTransform + cv2.warpAffine); None when every
        landmark is zero.  Channel order is kept (the reference passes BGR, the warp is per channel)."""
        import torch
        from .align import align_faces
        try:
            dev = self.model.device if self.model is not None else torch.device("cuda", _device_index(self.device))
            x = torch.as_tensor(np.ascontiguousarray(image, dtype=np.uint8))[None].to(dev)
            crops, ok = align_faces(x, [landmarks])
            return crops[0].cpu().numpy() if ok[0] else None
        except Exception as e:
            print(f"Loi align face: {e}")
            return None

    def detect_and_align(self, img_input):
        """Detect (device MTCNN) and align the largest confident face: PIL RGB 112 x 112, the margin crop
        when the face has no landmarks, or None (reference :206-242)."""
        from PIL import Image
        if self.face_detector is None:
            return None
        try:
            if isinstance(img_input, str):
                rgb = np.asarray(Image.open(img_input).convert("RGB"), dtype=np.uint8)
            elif isinstance(img_input, Image.Image):
                rgb = np.asarray(img_input.convert("RGB"), dtype=np.uint8)
            else:  # numpy BGR, as the reference's cv2 images
                rgb = np.ascontiguousarray(np.asarray(img_input, dtype=np.uint8)[..., ::-1])
        except Exception:
            return None
        det = self.face_detector.detect_rgb(rgb)
        if det is None:
            return None
        lm = det.get("landmarks")
        if lm:
            aligned = self.align_face(rgb, lm)
            if aligned is not None:
                return Image.fromarray(aligned)
        cropped = self.face_detector.crop_face(np.ascontiguousarray(rgb[..., ::-1]), margin=0.2, target_size=(112, 112))
        return Image.fromarray(np.ascontiguousarray(cropped[..., ::-1])) if cropped is not None else None

    def _detected(self, img_input):
        """The image the embedding is taken from: the aligned face when detection is on and finds one
        (reference extract_embedding :256-263), else the input."""
        if self.use_face_detection and self.face_detector is not None:
            aligned = self.detect_and_align(img_input)
            if aligned is not None:
                return aligned
        return img_input

    def _db_gallery(self):
        """Device copies of the dict db for cosine_similarity semantics (recognition_engine.py:41-63):
        a pair scores dot(a, b) when BOTH norms are within 1e-3 of 1, else dot / (|a| |b|).  A row's
        divisor therefore depends on the probe, so the rows are kept as
          'on'  — the rows whose norm is within 1e-3 of 1, raw (scored against unit-ish probes as is);
          'off' — the other rows divided by their norm (zero rows stay zero: score 0.0);
          'all' — every row divided by its norm (for probes that are not unit-ish), built on first use.
        A dict db of normalized embeddings (build_db, add_to_db) has no 'off' rows, and unit-ish probes
        (every fr_embed output) then take one search."""
        from .gallery import DeviceGallery
        key = (id(self._db), self._db.version)
        if self._g is not None and self._g[0] != key and self._g[0][0] == id(self._db):
            keys = self._db.journal_since(self._g[0][1])
            if keys is not None and self._db_apply_journal(keys):
                self._g = (key, self._g[1], self._g[2])
        if self._g is None or self._g[0] != key:
            names = list(self._db.keys())
            rows = np.stack([np.asarray(v, dtype=np.float32).reshape(-1) for v in self._db.values()])
            n = np.linalg.norm(rows, axis=1)
            on = np.abs(n - 1.0) < 1e-3
            dev = self.model.device.index if self.model is not None else _device_index(self.device)
            unit = rows / np.where(n > 0, n, 1.0)[:, None]
            parts = {"dev": dev, "dim": rows.shape[1], "pos": {k: i for i, k in enumerate(names)},
                     "on_mask": _Grow(on)}
            for tag, mask, src in (("on", on, rows), ("off", ~on, unit)):
                idx = np.nonzero(mask)[0]
                parts[tag] = (DeviceGallery(src[idx], dim=rows.shape[1], device=dev), _Grow(idx)) if len(idx) else None
            self._g = (key, parts, names)
        return self._g[1], self._g[2]

    def _db_apply_journal(self, keys) -> bool:
        """Apply the db's journaled assignments since this engine's copy synced (`keys`) to the device
        copy in place: a new name appends one row to its part (and to the 'all' copy), a re-assigned
        name overwrites its row when its norm class ('on' / 'off') is unchanged.  False (-> rebuild)
        for anything else."""
        from .gallery import DeviceGallery
        parts, names = self._g[1], self._g[2]
        for k in keys:
            v = np.asarray(self._db[k], dtype=np.float32).reshape(1, -1)
            if v.shape[1] != parts["dim"]:
                return False
            nv = float(np.linalg.norm(v))
            on = abs(nv - 1.0) < 1e-3
            u = v / (nv if nv > 0 else 1.0)
            tag = "on" if on else "off"
            src = v if on else u
            if k in parts["pos"]:
                i = parts["pos"][k]
                if bool(parts["on_mask"].view[i]) != on:
                    return False
                g, idx = parts[tag]
                g.update(int(np.searchsorted(idx.view, i)), src)
                if "all" in parts:
                    parts["all"][0].update(i, u)
            else:
                i = len(names)
                names.append(k)
                parts["pos"][k] = i
                parts["on_mask"].append(on)
                if parts[tag] is None:
                    parts[tag] = (DeviceGallery(src, dim=parts["dim"], device=parts["dev"]), _Grow(np.array([i])))
                else:
                    g, idx = parts[tag]
                    g.add(src)
                    idx.append(i)
                if "all" in parts:
                    g, idx = parts["all"]
                    g.add(u)
                    idx.append(i)
        return True

    # ------------------------------------------------------------------ embedding
    # ------------------------------------------------------------------ embedding
    def extract_embedding(self, img_input) -> Optional[np.ndarray]:
        if self.model is None:
            print("Model chua duoc load")
            return None
        return extract_embedding_single(self._detected(img_input), self.model, self.transform, self.device)

    # ------------------------------------------------------------------ matching
    @staticmethod
    def _search_mapped(part, P, k):
        """Top-k of host probes P against one device part; indices mapped to db rows."""
        import torch
        g, idx = part
        s, i = g.search_device(torch.from_numpy(np.ascontiguousarray(P)).to(g.device), min(k, g.ntotal))
        return s.cpu().numpy(), idx.view[i.cpu().numpy()]

    @staticmethod
    def _merge(lists, k):
        """(score desc, db row asc) merge of per-part top-k lists — the stable sort's order."""
        s = np.concatenate([a for a, _ in lists], 1)
        i = np.concatenate([b for _, b in lists], 1)
        order = np.lexsort((i, -s), axis=1)[:, :k]
        return np.take_along_axis(s, order, 1), np.take_along_axis(i, order, 1)

    def _db_topk(self, E: np.ndarray, k: int):
        """Top-k db rows of every probe in cosine_similarity semantics (see _db_gallery)."""
        parts, names = self._db_gallery()
        k = min(k, len(names))
        E = np.asarray(E, dtype=np.float32).reshape(len(E), -1)
        npr = np.linalg.norm(E, axis=1)
        p_on = np.abs(npr - 1.0) < 1e-3
        E_unit = E / np.where(npr > 0, npr, 1.0)[:, None]
        S = np.zeros((len(E), k), np.float32)
        I = np.zeros((len(E), k), np.int64)
        sel = np.nonzero(p_on)[0]
        if len(sel):  # unit-ish probes: raw against 'on' rows, dot / (|p| |g|) against 'off' rows
            lists = []
            if parts["on"] is not None:
                lists.append(self._search_mapped(parts["on"], E[sel], k))
            if parts["off"] is not None:
                lists.append(self._search_mapped(parts["off"], E_unit[sel], k))
            S[sel], I[sel] = self._merge(lists, k) if len(lists) > 1 else lists[0]
        sel = np.nonzero(~p_on)[0]
        if len(sel):  # other probes (zero probes stay zero: every score 0.0): dot / (|p| |g|) everywhere
            if "all" not in parts:
                from .gallery import DeviceGallery
                rows = np.stack([np.asarray(self._db[nm], dtype=np.float32).reshape(-1) for nm in names])
                nr = np.linalg.norm(rows, axis=1)
                parts["all"] = (DeviceGallery(rows / np.where(nr > 0, nr, 1.0)[:, None], dim=parts["dim"],
                                              device=parts["dev"]), _Grow(np.arange(len(names))))
            S[sel], I[sel] = self._search_mapped(parts["all"], E_unit[sel], k)
        return S, I, names

    def _result_db(self, s_row, i_row, names):
        top = [(names[j], float(v)) for v, j in zip(s_row, i_row)]
        best_name, best_score = top[0]
        if best_score < self.threshold:
            return "Unknown", best_score, top
        return best_name, best_score, top

    def recognize_with_db(self, embedding: np.ndarray) -> Tuple[str, float, List[Tuple[str, float]]]:
        if self.db is None:
            return "No database", 0.0, []
        s, i, names = self._db_topk(np.asarray(embedding)[None], 5)
        return self._result_db(s[0], i[0], names)

    def _faiss_topk(self, E: np.ndarray, k: int):
        import torch
        if k > MAX_K:
            raise ValueError(f"k={k} > {MAX_K} is not supported by fr_match_topk")
        E = np.asarray(E, dtype=np.float32).reshape(len(E), -1)
        E = E / (np.linalg.norm(E, axis=1, keepdims=True) + 1e-8)
        P = torch.from_numpy(np.ascontiguousarray(E)).to(self.faiss_index.device)
        s, i = self.faiss_index.search_device(P, k)
        return s.cpu().numpy(), i.cpu().numpy()

    def _result_faiss(self, s_row, i_row):
        results = []
        for idx, score in zip(i_row, s_row):
            if idx == -1:
                continue
            name = self.id_to_label.get(int(idx), f"ID_{idx}") if self.id_to_label else f"ID_{idx}"
            results.append((name, float(score)))
        if not results:
            return "Unknown", 0.0, []
        best_name, best_score = results[0]
        if best_score < self.threshold:
            return "Unknown", best_score, results
        return best_name, best_score, results

    def recognize_with_faiss(self, embedding: np.ndarray, k: int = 5) -> Tuple[str, float, List[Tuple[str, float]]]:
        if self.faiss_index is None:
            return "No FAISS index", 0.0, []
        s, i = self._faiss_topk(np.asarray(embedding)[None], k)
        return self._result_faiss(s[0], i[0])

    # ------------------------------------------------------------------ end-to-end
    def recognize(self, img_input, use_faiss: bool = None, k: int = 5) -> Dict:
        return self.recognize_batch([img_input], use_faiss, k)[0]

    def recognize_batch(self, img_inputs: List, use_faiss: bool = None, k: int = 5) -> List[Dict]:
        results = [{"identity": "Unknown", "confidence": 0.0, "top_k": [], "embedding": None, "status": "success"}
                   for _ in img_inputs]
        ok, crops = [], []
        if self.model is not None:
            for n, img in enumerate(img_inputs):
                try:
                    crops.append(_load_u8(self._detected(img), self.transform))
                    ok.append(n)
                except Exception as e:
                    if isinstance(img, str):
                        print(f"Loi xu ly {img}: {e}")
        else:
            print("Model chua duoc load")
        for n in range(len(img_inputs)):
            if n not in ok:
                results[n]["status"] = "error"
                results[n]["message"] = "Cannot extract embedding (no face or invalid image)"
        if not ok:
            return results
        E = _embed_u8(self.model, crops)  # device resize + fr_embed in 256-image batches
        if use_faiss is None:
            use_faiss = self.faiss_index is not None
        if use_faiss and self.faiss_index is not None:
            s, i = self._faiss_topk(E, k)
            ident = [self._result_faiss(s[r], i[r]) for r in range(len(ok))]
        elif self.db is not None:
            s, i, names = self._db_topk(E, 5)
            ident = [self._result_db(s[r], i[r], names) for r in range(len(ok))]
        else:
            for r, n in enumerate(ok):
                results[n]["embedding"] = E[r]
                results[n]["status"] = "error"
                results[n]["message"] = "No database loaded"
            return results
        for r, n in enumerate(ok):
            results[n]["embedding"] = E[r].astype(np.float32)
            results[n]["identity"], results[n]["confidence"], results[n]["top_k"] = ident[r]
        return results

    def add_to_db(self, name: str, img_inputs: List) -> bool:
        crops = []
        if self.model is not None:
            for img in img_inputs:
                try:
                    crops.append(_load_u8(self._detected(img), self.transform))
                except Exception as e:
                    if isinstance(img, str):
                        print(f"Loi xu ly {img}: {e}")
        if not crops:
            print(f"Khong the extract embedding cho {name}")
            return False
        m = segment_means(self.model, [crops])[0]  # fr_embed + fr_segment_mean_normalize (:411-413)
        if self.db is None:
            self.db = {}
        self.db[name] = m
        print(f"Added {name} to database (from {len(crops)} images)")
        return True

    def save_db(self, path: str):
        if self.db:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            np.save(path, dict(self.db))
            print(f"Saved database: {path}")

    def get_db_identities(self) -> List[str]:
        return list(self.db.keys()) if self.db else []



class FaceNetMatcher:
    """The FaceNet web route's matcher (web_app.py:537-559) on the device: the probe and every db row are
    divided by (|v| + 1e-8) (the route renormalizes rows in case the db was not normalized), score = dot
    product (fr_match_topk, (score desc, row asc) = the stable sort), distance = |e - row| computed for
    the returned rows exactly as the route does, best < threshold -> "Unknown".  One device gallery per
    db, rebuilt when the dict changes (same tracking as RecognitionEngine)."""

    def __init__(self, db: Dict[str, np.ndarray], threshold: float = 0.5, device: int = 0):
        from .gallery import DeviceGallery
        self.threshold = threshold
        self.names = list(db.keys())
        rows = np.stack([np.asarray(v, dtype=np.float32).reshape(-1) for v in db.values()])
        self.rows = rows / (np.linalg.norm(rows, axis=1, keepdims=True) + 1e-8)
        self.gallery = DeviceGallery(self.rows, dim=rows.shape[1], device=device)

    def match_batch(self, embeddings: np.ndarray, k: int = 5) -> List[Dict]:
        import torch
        E = np.asarray(embeddings, dtype=np.float32).reshape(len(embeddings), -1)
        E = E / (np.linalg.norm(E, axis=1, keepdims=True) + 1e-8)
        k = min(k, len(self.names))
        s, i = self.gallery.search_device(torch.from_numpy(np.ascontiguousarray(E)).to(self.gallery.device), k)
        s, i = s.cpu().numpy(), i.cpu().numpy()
        out = []
        for r in range(len(E)):
            top = [(self.names[j], float(v), float(np.linalg.norm(E[r] - self.rows[j]))) for v, j in zip(s[r], i[r])]
            name, score, dist = top[0]
            out.append({"identity": "Unknown" if score < self.threshold else name, "confidence": score,
                        "distance": dist, "top_k": top, "status": "success"})
        return out

    def match(self, embedding: np.ndarray, k: int = 5) -> Dict:
        return self.match_batch(np.asarray(embedding)[None], k)[0]


def create_engine_from_embeddings_dir(model_path: str, embeddings_dir: str, threshold: float = 0.5,
                                      device: str = None) -> RecognitionEngine:
    idx = os.path.join(embeddings_dir, "arcface_index.faiss")  # recognition_engine.py:453
    if not os.path.exists(idx) and os.path.exists(os.path.join(embeddings_dir, "arcface_index.npz")):
        idx = os.path.join(embeddings_dir, "arcface_index.npz")  # round-1 row files
    protos = os.path.join(embeddings_dir, "arcface_prototypes.npy")
    mapping = os.path.join(embeddings_dir, "label_mapping.npy")
    return RecognitionEngine(model_path=model_path, faiss_index_path=idx if os.path.exists(idx) else None,
                             prototypes_path=protos if os.path.exists(protos) else None,
                             label_mapping_path=mapping if os.path.exists(mapping) else None,
                             threshold=threshold, device=device)


# The north star names "UnifiedRecognitionEngine"; the reference's README calls recognition_engine.py the
# "Unified Recognition Engine" (README.md:202) but the class is RecognitionEngine (SURVEY.md §0 note 3).
UnifiedRecognitionEngine = RecognitionEngine
