"""Drop-in for the reference's ``inference/extract_embeddings.py`` (same names, arguments, return
values and error conventions), with every forward pass and every gallery reduction on the MI355X
through libfrhip.so.

Reference → here:
  load_arcface_model  :80-123   checkpoint schema read with torch.load(weights_only=True); arch
                                 auto-detected (ResNet-50 ArcFace / IResNet100 / InceptionResnetV1)
  load_facenet_model  :126-167  FaceNet state_dict (model.* / backbone.* prefixes, logits ignored)
  get_transform / get_facenet_transform :170-185   Resize(PIL bilinear)+ToTensor+Normalize(0.5)
  extract_embedding_single :348-389   one image → np.f32 [512] or None on any error
  extract_embeddings_batch :392-443   (emb [M,512], valid_paths); bad files skipped; empty → (array([]), [])
  extract_embedding_for_folder :714-762   per-identity mean + renorm on the device (segment_means: batched
                                 fr_embed + fr_segment_mean_normalize) instead of one forward per image
  build_db :765-835              every identity's crops in shared 256-image fr_embed batches, one
                                 segmented-mean launch per ~4096 images
  compute_prototypes :555-592 / build_faiss_index :595-645 (→ DeviceGallery, IndexFlatIP surface; the
                                 .faiss flat-index file format without faiss: faiss_io.py)
  build_db :765-835, extract_embeddings_from_csv :446-552, full_pipeline :838-888
  FacePreprocessor / FaceNetPreprocessor :188-345   device MTCNN + device alignment warp (face_detector.py,
                                 SURVEY.md §8f row 4); without MTCNN weights the raw image is used, as the
                                 reference does when its detector is unavailable.  t-SNE plotting is out of
                                 scope.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import weights as Wt

# Host/device memory bounds of the batched paths: decoded images stay at full resolution
# until the device resize, so build_db flushes by decoded bytes as well as by image count, and one
# _device_crops upload carries at most UPLOAD_BYTES of decoded pixels.
FLUSH_IMAGES = 4096
FLUSH_BYTES = 1 << 30
UPLOAD_BYTES = 256 << 20
ARCFACE_TEMPLATE = np.array([[38.2946, 51.6963], [73.5318, 51.5014], [56.0252, 71.7366],
                             [41.5493, 92.3655], [70.7299, 92.2041]], dtype=np.float32)
IMG_EXTS = (".jpg", ".jpeg", ".png", ".webp")


def _device_index(device) -> int:
    """'cuda', 'cuda:1', torch.device or int → HIP device index.  There is no CPU path."""
    if device is None:
        return 0
    if isinstance(device, int):
        return device
    s = str(device)
    if s.startswith("cuda"):
        return int(s.split(":")[1]) if ":" in s else 0
    raise ValueError(f"device {device!r}: facerecognition_amd runs on a ROCm GPU ('cuda[:N]'); "
                     "there is deliberately no CPU fallback")


# ---------------------------------------------------------------------------------------- models
def load_arcface_model(model_path: str, device: str = "cuda"):
    """Returns (model, info) like the reference; model(x, labels=None) → un-normalized embedding."""
    from .model import FRModel

    if not os.path.exists(model_path):
        raise FileNotFoundError(f"Model khong ton tai: {model_path}")
    sd, ck = Wt.load_checkpoint(model_path)
    arch = Wt.detect_arch(sd)
    config = ck.get("config") or {}
    num_classes = config.get("num_classes", ck.get("num_classes") or 100)
    embedding_size = (config.get("model") or {}).get("embedding_size", 512)
    model = FRModel(arch, sd, device=_device_index(device))
    info = {"num_classes": num_classes, "embedding_size": embedding_size, "arch": arch,
            "epoch": ck.get("epoch") if ck.get("epoch") is not None else "N/A",
            "val_acc": ck.get("val_acc") if ck.get("val_acc") is not None else "N/A",
            "best_val_acc": ck.get("best_val_acc") if ck.get("best_val_acc") is not None else "N/A"}
    print(f"Loaded model from {model_path} ({arch}, {model.dtype})")
    return model, info


def load_facenet_model(model_path: str, device: str = "cuda"):
    model, info = load_arcface_model(model_path, device)
    if model.arch != "irv1_facenet":
        raise ValueError(f"{model_path} is not an InceptionResnetV1 (FaceNet) checkpoint ({model.arch})")
    return model, {k: info[k] for k in ("embedding_size", "epoch", "best_val_acc")}


# ---------------------------------------------------------------------------------------- transforms
class _Transform:
    """Resize((S,S)) with PIL bilinear (identity when already S x S) + ToTensor + Normalize(0.5, 0.5)."""

    def __init__(self, image_size: int):
        self.size = image_size

    def resize(self, img):
        from PIL import Image
        img = img.convert("RGB")
        if img.size != (self.size, self.size):
            img = img.resize((self.size, self.size), Image.BILINEAR)
        return img

    def __call__(self, img):
        import torch
        a = np.asarray(self.resize(img), dtype=np.uint8)
        t = torch.from_numpy(a.copy()).permute(2, 0, 1).contiguous().float().div(255)
        return (t - 0.5) / 0.5


def get_transform(image_size: int = 112):
    return _Transform(image_size)


def get_facenet_transform(image_size: int = 160):
    return _Transform(image_size)


def _load_u8(img_input, transform) -> np.ndarray:
    """PIL/path -> decoded RGB u8 HWC at its own size (the Resize of the transform runs on the device:
    _device_crops; ToTensor + Normalize are fused into fr_embed's u8 path)."""
    from PIL import Image
    if not isinstance(transform, _Transform):
        raise TypeError("transform must come from get_transform()/get_facenet_transform()")
    img = Image.open(img_input) if isinstance(img_input, str) else img_input
    return np.asarray(img.convert("RGB"), dtype=np.uint8)


def _check_transform(model, transform) -> None:
    """The transform's Resize target must be the model's input side (the reference resizes to the
    transform's image_size: get_transform / get_facenet_transform, extract_embeddings.py:170-185)."""
    if not isinstance(transform, _Transform):
        raise TypeError("transform must come from get_transform()/get_facenet_transform()")
    if transform.size != model.input_size:
        raise ValueError(f"transform resizes to {transform.size}x{transform.size} but the {model.arch} model "
                         f"takes {model.input_size}x{model.input_size} crops")


def _device_crops(arrays: List[np.ndarray], size: int, device):
    """Decoded RGB u8 images of any sizes -> device u8 [n, size, size, 3]: images already size x size are
    copied, the others go through fr_resize_u8 (Pillow's BILINEAR resize, bit-exact), one launch per
    distinct input size and upload of at most UPLOAD_BYTES decoded bytes (large photos are not staged
    256 at a time)."""
    import torch
    from .align import resize_u8
    out = torch.empty((len(arrays), size, size, 3), dtype=torch.uint8, device=device)
    by_shape: Dict[tuple, List[int]] = {}
    for i, a in enumerate(arrays):
        by_shape.setdefault(a.shape, []).append(i)
    for shape, idx in by_shape.items():
        per = max(1, UPLOAD_BYTES // max(1, int(np.prod(shape))))
        for c in range(0, len(idx), per):
            part = idx[c:c + per]
            x = torch.from_numpy(np.ascontiguousarray(np.stack([arrays[i] for i in part]))).to(device, non_blocking=True)
            if shape[:2] != (size, size):
                x = resize_u8(x, size, size)
            out[torch.as_tensor(part, device=device)] = x
    return out


def _embed_u8(model, arrays) -> np.ndarray:
    """Normalized embeddings (host f32 [n, D]) of decoded images of any sizes, in batches of up to
    model.max_batch (256), resized on the device."""
    import torch
    mb = max(1, getattr(model, "max_batch", 0) or 256)
    arrays = list(arrays)
    outs = []
    for a in range(0, len(arrays), mb):
        x = _device_crops(arrays[a:a + mb], model.input_size, model.device)
        outs.append(model.embed(x, normalize=True).cpu().numpy())
    return np.concatenate(outs) if outs else np.zeros((0, model.embedding_size), np.float32)


# ---------------------------------------------------------------------------------------- extraction
def extract_embedding_single(img_input, model, transform, device: str = "cuda",
                             model_type: str = "arcface") -> Optional[np.ndarray]:
    try:
        _check_transform(model, transform)
        u8 = _load_u8(img_input, transform)
        return _embed_u8(model, [u8])[0].astype(np.float32).flatten()
    except Exception as e:  # reference: any failure → None (extract_embeddings.py:386-389)
        if isinstance(img_input, str):
            print(f"Loi xu ly {img_input}: {e}")
        return None


def extract_embeddings_batch(image_paths: List[str], model, transform, device: str = "cuda",
                             batch_size: int = 64, model_type: str = "arcface") -> Tuple[np.ndarray, List[str]]:
    embeddings, valid_paths = [], []
    for i in range(0, len(image_paths), batch_size):
        imgs, paths = [], []
        for path in image_paths[i:i + batch_size]:
            try:
                imgs.append(_load_u8(path, transform))
                paths.append(path)
            except Exception as e:
                print(f"Skip {path}: {e}")
        if not imgs:
            continue
        _check_transform(model, transform)
        embeddings.append(_embed_u8(model, imgs))
        valid_paths.extend(paths)
    if not embeddings:
        return np.array([]), []
    return np.vstack(embeddings).astype(np.float32), valid_paths


def segment_means(model, groups: List[List[np.ndarray]]) -> List[Optional[np.ndarray]]:
    """Identity rows of a gallery, batched on the device: every decoded image of every
    group (any size: resized on the device) goes through fr_embed in batches of up to model.max_batch (256) images into one device buffer, and
    fr_segment_mean_normalize reduces each group to mean / (||mean|| + 1e-8) -- the reference's per-folder
    ``np.mean`` + renorm (extract_embeddings.py:755-760, recognition_engine.py:411-413), for all groups
    in one launch.  Empty groups give None (the reference skips an identity with no valid image)."""
    import torch
    from . import _native as N
    out: List[Optional[np.ndarray]] = [None] * len(groups)
    live = [g for g, imgs in enumerate(groups) if len(imgs)]
    if not live:
        return out
    crops = [c for g in live for c in groups[g]]
    dev = model.device
    D = model.embedding_size
    E = torch.empty((len(crops), D), dtype=torch.float32, device=dev)
    mb = max(1, getattr(model, "max_batch", 0) or 256)
    for a in range(0, len(crops), mb):
        x = _device_crops(crops[a:a + mb], model.input_size, dev)
        model.embed(x, normalize=True, out=E[a:a + len(x)])
    starts = np.cumsum([0] + [len(groups[g]) for g in live]).astype(np.int32)
    seg = torch.from_numpy(starts).to(dev)
    M = torch.empty((len(live), D), dtype=torch.float32, device=dev)
    N.check(N.lib().fr_segment_mean_normalize(N.ptr(E), D, N.ptr(seg), len(live), N.ptr(M), N.stream_ptr(dev)),
            "fr_segment_mean_normalize")
    rows = M.cpu().numpy()
    for r, g in enumerate(live):
        out[g] = rows[r]
    return out


class FacePreprocessor:
    """Detect + align before embedding (reference :188-280): the device MTCNN (face_detector.FaceDetector,
    confidence 0.9, largest face) and the device 5-point warp to ARCFACE_TEMPLATE; the margin crop when a
    face has no landmarks.  Without MTCNN weights the detector is None and ``process`` returns the raw
    image, as the reference does without facenet-pytorch."""

    out_size = 112

    def __init__(self, device: str = "cuda", weights_dir: str = None, detector=None):
        self.device = device
        self.detector = detector
        if self.detector is None:
            try:
                from .face_detector import FaceDetector
                self.detector = FaceDetector(backend="mtcnn", device=device, confidence_threshold=0.9,
                                             select_largest=True, weights_dir=weights_dir)
                print(f"[OK] {type(self).__name__} initialized (MTCNN)")
            except Exception as e:
                print(f"[WARN] Khong the khoi tao Face Detector: {e}")
                self.detector = None

    def _raw(self, rgb):
        from PIL import Image
        return Image.fromarray(rgb)

    def _face(self, rgb, det):
        from PIL import Image
        from .align import align_faces
        import torch
        lm = det.get("landmarks")
        if lm:
            x = torch.as_tensor(np.ascontiguousarray(rgb))[None].to(self.detector.detector.device)
            crops, ok = align_faces(x, [lm])
            if ok[0]:
                return Image.fromarray(crops[0].cpu().numpy())
        return self._crop(rgb)

    def _crop(self, rgb):
        from PIL import Image
        c = self.detector.crop_face(np.ascontiguousarray(rgb[..., ::-1]), margin=0.2,
                                    target_size=(self.out_size, self.out_size))
        return Image.fromarray(np.ascontiguousarray(c[..., ::-1])) if c is not None else None

    def process(self, img_input):
        """Path or BGR u8 array -> PIL RGB face (or the raw image without a detector), None if no face."""
        from PIL import Image
        if isinstance(img_input, str):
            rgb = np.asarray(Image.open(img_input).convert("RGB"), dtype=np.uint8)
        else:
            rgb = np.ascontiguousarray(np.asarray(img_input, dtype=np.uint8)[..., ::-1])
        if self.detector is None:
            return self._raw(rgb)
        det = self.detector.detect_rgb(rgb)
        return None if det is None else self._face(rgb, det)


class FaceNetPreprocessor(FacePreprocessor):
    """FaceNet's detect + crop (reference :283-345): the margin-0.2 crop resized to 160 x 160 (no alignment);
    without a detector the raw image resized to 160 x 160."""

    out_size = 160

    def _raw(self, rgb):
        from PIL import Image
        return Image.fromarray(rgb).resize((160, 160))

    def _face(self, rgb, det):
        return self._crop(rgb)


def _folder_crops(folder: str, transform, preprocessor=None) -> List[np.ndarray]:
    paths = [os.path.join(folder, f) for f in os.listdir(folder) if f.lower().endswith(IMG_EXTS)]
    imgs = []
    for p in paths:  # os.listdir order, as the reference
        try:
            face = preprocessor.process(p) if preprocessor is not None else None  # reference :744-749
            imgs.append(_load_u8(face if face is not None else p, transform))
        except Exception as e:
            print(f"Loi xu ly {p}: {e}")
    return imgs


def extract_embedding_for_folder(folder: str, model, transform, device: str = "cuda", preprocessor=None,
                                 model_type: str = "arcface") -> Optional[np.ndarray]:
    if not os.path.exists(folder):
        return None
    _check_transform(model, transform)
    return segment_means(model, [_folder_crops(folder, transform, preprocessor)])[0]


def compute_prototypes(embeddings: np.ndarray, labels: np.ndarray, output_path: str = None) -> np.ndarray:
    print("\n=== COMPUTING PROTOTYPES ===")
    unique_labels = np.unique(labels)
    prototypes = np.zeros((len(unique_labels), embeddings.shape[1]), dtype=np.float32)
    for label in unique_labels:
        p = embeddings[labels == label].mean(axis=0)
        prototypes[label] = p / (np.linalg.norm(p) + 1e-8)
    print(f"Computed {len(unique_labels)} prototypes")
    if output_path:
        np.save(output_path, prototypes)
        print(f"Saved prototypes: {output_path}")
    return prototypes


def build_faiss_index(embeddings: np.ndarray, output_path: str = None, use_gpu: bool = True):
    """IndexFlatIP equivalent on the GPU: rows L2-normalized (+1e-8) like the reference; saved in FAISS's
    own flat-index file format (faiss_io.write_flat_index), readable by faiss.read_index and by
    read_index here."""
    from .faiss_io import write_flat_index
    from .gallery import DeviceGallery

    print("\n=== BUILDING DEVICE INDEX (IndexFlatIP semantics) ===")
    e = np.asarray(embeddings, dtype=np.float32)
    e = e / (np.linalg.norm(e, axis=1, keepdims=True) + 1e-8)
    index = DeviceGallery(e, dim=e.shape[1])
    print(f"Index built: {index.ntotal} vectors, {e.shape[1]}D")
    if output_path:
        write_flat_index(output_path, e)
        print(f"Saved FAISS index: {output_path}")
    return index


def read_index(path: str):
    """faiss.read_index for flat indexes (the reference's arcface_index.faiss) into a DeviceGallery with
    IndexFlatIP search semantics; round-1 .npz row files are still accepted."""
    from .faiss_io import read_flat_index
    from .gallery import DeviceGallery
    if path.endswith(".npz") or (not os.path.exists(path) and os.path.exists(path + ".npz")):
        with np.load(path if os.path.exists(path) else path + ".npz", allow_pickle=False) as z:
            rows = z["rows"]
    else:
        rows, metric = read_flat_index(path)
        if metric != 0:
            raise ValueError(f"{path}: metric {metric} index; the reference builds IndexFlatIP (metric 0)")
    return DeviceGallery(rows, dim=rows.shape[1])


def visualize_tsne(*_a, **_k):
    raise NotImplementedError("t-SNE plotting is out of scope for facerecognition_amd (SURVEY.md §2.1 row 1)")


# ---------------------------------------------------------------------------------------- drivers
def build_db(model_path: str, root_folder: str = "data/celeb", save_path: str = "data/arcface_embeddings_db.npy",
             device: str = None, use_face_detection: bool = True, model_type: str = "arcface") -> None:
    print("=" * 60)
    print(f"EXTRACT EMBEDDINGS DATABASE ({model_type.upper()})")
    print("=" * 60)
    device = device or "cuda"
    if not os.path.exists(root_folder):
        print(f"Root folder khong ton tai: {root_folder}")
        return
    if model_type == "facenet":
        model, _ = load_facenet_model(model_path, device)
        transform = get_facenet_transform()
    else:
        model, _ = load_arcface_model(model_path, device)
        transform = get_transform(Wt.INPUT_SIZE[model.arch])
    preprocessor = None
    if use_face_detection:  # reference :800-805
        preprocessor = (FaceNetPreprocessor if model_type == "facenet" else FacePreprocessor)(device=device)
    db: Dict[str, np.ndarray] = {}
    persons = [p for p in os.listdir(root_folder) if os.path.isdir(os.path.join(root_folder, p))]
    print(f"\nTim thay {len(persons)} celebrities")
    # identities are embedded together: crops of consecutive persons are collected
    # until FLUSH_IMAGES images or FLUSH_BYTES decoded bytes, then embedded in 256-image fr_embed batches
    # and reduced per person by one segmented-mean launch; host memory stays bounded by one flush
    pending: List[str] = []
    groups: List[List[np.ndarray]] = []

    def flush():
        for person, emb in zip(pending, segment_means(model, groups)):
            if emb is not None:
                db[person] = emb
        pending.clear()
        groups.clear()

    for person in persons:
        pending.append(person)
        groups.append(_folder_crops(os.path.join(root_folder, person), transform, preprocessor))
        if sum(len(g) for g in groups) >= FLUSH_IMAGES or sum(a.nbytes for g in groups for a in g) >= FLUSH_BYTES:
            flush()
    flush()
    if not db:
        print("\nKhong co embeddings nao duoc tao!")
        return
    os.makedirs(os.path.dirname(save_path) or ".", exist_ok=True)
    np.save(save_path, db)
    print(f"\nDa luu {len(db)} embeddings vao {save_path}")
    print(f"Success rate: {len(db)}/{len(persons)} ({100 * len(db) / len(persons):.1f}%)")


def extract_embeddings_from_csv(model_path: str, csv_path: str, data_root: str = None,
                                output_dir: str = "data/embeddings", device: str = None, batch_size: int = 64) -> Dict:
    import pandas as pd

    os.makedirs(output_dir, exist_ok=True)
    model, _ = load_arcface_model(model_path, device or "cuda")
    transform = get_transform(Wt.INPUT_SIZE[model.arch])
    df = pd.read_csv(csv_path)
    path_col = "image_path" if "image_path" in df.columns else ("image" if "image" in df.columns else None)
    id_col = "identity_name" if "identity_name" in df.columns else ("person_id" if "person_id" in df.columns else None)
    if path_col is None:
        raise ValueError(f"CSV khong co cot path. Columns: {list(df.columns)}")
    if id_col is None:
        raise ValueError(f"CSV khong co cot identity. Columns: {list(df.columns)}")
    image_paths = [os.path.join(data_root, p) for p in df[path_col]] if data_root else df[path_col].tolist()
    identities = df[id_col].astype(str).tolist()
    unique_ids = sorted(set(identities))
    id_to_label = {id_: i for i, id_ in enumerate(unique_ids)}
    labels = [id_to_label[i] for i in identities]
    embeddings, valid_paths = extract_embeddings_batch(image_paths, model, transform, device, batch_size)
    index_of = {p: i for i, p in enumerate(image_paths)}
    valid_idx = [index_of[p] for p in valid_paths]
    valid_labels = [labels[i] for i in valid_idx]
    valid_ids = [identities[i] for i in valid_idx]
    np.save(os.path.join(output_dir, "arcface_train_embeddings.npy"), embeddings)
    pd.DataFrame({"image_path": valid_paths, "identity": valid_ids, "label": valid_labels}).to_csv(
        os.path.join(output_dir, "embeddings_metadata.csv"), index=False)
    np.save(os.path.join(output_dir, "label_mapping.npy"),
            {"id_to_label": id_to_label, "label_to_id": {v: k for k, v in id_to_label.items()}})
    return {"embeddings": embeddings, "labels": np.array(valid_labels), "identities": valid_ids,
            "paths": valid_paths, "id_to_label": id_to_label}


def full_pipeline(model_path: str, csv_path: str, data_root: str = None, output_dir: str = "data/embeddings",
                  device: str = None, batch_size: int = 64):
    result = extract_embeddings_from_csv(model_path, csv_path, data_root, output_dir, device, batch_size)
    prototypes = compute_prototypes(result["embeddings"], result["labels"],
                                    os.path.join(output_dir, "arcface_prototypes.npy"))
    build_faiss_index(prototypes, os.path.join(output_dir, "arcface_index.faiss"))
    print("t-SNE visualization skipped (out of scope)")
    return result


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="Extract embeddings (MI355X)")
    ap.add_argument("--model-path", default="models/checkpoints/arcface/arcface_best.pth")
    ap.add_argument("--mode", choices=["db", "csv", "full"], default="full")
    ap.add_argument("--csv-path", default=None)
    ap.add_argument("--data-root", default=None)
    ap.add_argument("--data-dir", default="data/celeb")
    ap.add_argument("--output-dir", default="data/embeddings")
    ap.add_argument("--output-path", default="data/arcface_embeddings_db.npy")
    ap.add_argument("--device", default=None)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--use-face-detection", action="store_true", default=True)
    ap.add_argument("--no-face-detection", action="store_true")
    ap.add_argument("--model-type", choices=["arcface", "facenet"], default="arcface")
    a = ap.parse_args(argv)
    use_fd = a.use_face_detection and not a.no_face_detection
    if a.mode == "db":
        build_db(a.model_path, a.data_dir, a.output_path, a.device, use_fd, a.model_type)
    elif a.csv_path is None:
        print("Vui long cung cap --csv-path")
    elif a.mode == "csv":
        extract_embeddings_from_csv(a.model_path, a.csv_path, a.data_root, a.output_dir, a.device, a.batch_size)
    else:
        full_pipeline(a.model_path, a.csv_path, a.data_root, a.output_dir, a.device, a.batch_size)


if __name__ == "__main__":
    main()
