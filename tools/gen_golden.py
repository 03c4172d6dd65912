#!/usr/bin/env python3
"""Generate the reference-pinned golden fixtures (run in the survey container, where
/root/reference exists; the GPU box never runs this).

It imports the reference's OWN code — models/arcface/arcface_model.py (ArcFaceModel),
inference/extract_embeddings.py (get_transform, extract_embedding_single, extract_embeddings_batch)
and inference/recognition_engine.py (cosine_similarity, RecognitionEngine.recognize_with_db) — with
shims only for modules that are not installed here:
  * torchvision.models.resnet50 -> oracle.models.ResNet50 (same module layout / state_dict keys)
  * torchvision.transforms      -> Compose / Resize (PIL bilinear) / ToTensor / Normalize
  * cv2                         -> empty module (imported at module top, unused on this path)
ArcFaceModel is built with pretrained=False (as evaluate_arcface_kaggle.ipynb cell 7 does) and
loaded with the synthetic weights of facerecognition_amd.weights.synth_state_dict.

Output: tests/golden/arcface_r50_golden.npz (data only — inputs and expected outputs).
"""
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, ROOT)

from facerecognition_amd import weights as W  # noqa: E402
from facerecognition_amd.synthetic import planted_gallery, synthetic_crops  # noqa: E402
from oracle import models as OM  # noqa: E402


def install_shims():
    from PIL import Image

    tv = types.ModuleType("torchvision")
    models = types.ModuleType("torchvision.models")

    def resnet50(pretrained=False, weights=None, **_k):
        if pretrained or weights is not None:
            raise RuntimeError("no network: pretrained torchvision weights are unavailable")
        return OM.ResNet50()

    models.resnet50 = resnet50
    tr = types.ModuleType("torchvision.transforms")

    class Compose:
        def __init__(self, ts):
            self.ts = ts

        def __call__(self, x):
            for t in self.ts:
                x = t(x)
            return x

    class Resize:
        def __init__(self, size):
            self.size = size

        def __call__(self, img):
            h, w = self.size
            return img if img.size == (w, h) else img.resize((w, h), Image.BILINEAR)

    class ToTensor:
        def __call__(self, img):
            a = torch.from_numpy(np.asarray(img, dtype=np.uint8).copy())
            return a.permute(2, 0, 1).contiguous().float().div(255)

    class Normalize:
        def __init__(self, mean, std):
            self.mean = torch.tensor(mean).view(-1, 1, 1)
            self.std = torch.tensor(std).view(-1, 1, 1)

        def __call__(self, t):
            return (t - self.mean) / self.std

    tr.Compose, tr.Resize, tr.ToTensor, tr.Normalize = Compose, Resize, ToTensor, Normalize
    tv.models, tv.transforms = models, tr
    sys.modules["torchvision"], sys.modules["torchvision.models"] = tv, models
    sys.modules["torchvision.transforms"] = tr
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))


def main(out=os.path.join(ROOT, "tests", "golden", "arcface_r50_golden.npz")):
    if not os.path.isdir(REF):
        raise SystemExit(f"{REF} not present: goldens are generated in the survey container only")
    torch.set_num_threads(os.cpu_count() or 1)
    install_shims()
    sys.path.insert(0, REF)
    import importlib.util

    from PIL import Image

    spec = importlib.util.spec_from_file_location("ref_arcface_model", os.path.join(REF, "models/arcface/arcface_model.py"))
    am = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(am)
    from inference import extract_embeddings as ee  # reference module (shimmed deps)
    from inference import recognition_engine as re_  # reference module

    num_classes = 100
    sd = W.synth_state_dict("resnet50_arcface", num_classes=num_classes)
    model = am.ArcFaceModel(num_classes=num_classes, embedding_size=512, pretrained=False)
    missing = model.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()}, strict=True)
    model.eval()
    transform = ee.get_transform()

    probes = synthetic_crops(8, 112, seed=0)
    # reference path per image: extract_embedding_single (PIL in -> np.f32 [512])
    single = np.stack([ee.extract_embedding_single(Image.fromarray(p), model, transform, "cpu") for p in probes])
    # batched path: model(x, labels=None) -> F.normalize, as in extract_embeddings_batch
    x = torch.stack([transform(Image.fromarray(p)) for p in probes])
    with torch.no_grad():
        raw = model(x, labels=None)
        batch = torch.nn.functional.normalize(raw, p=2, dim=1).numpy()
    # natural-image probe: the reference's own uploads/anh1.jpg through get_transform (PIL resize)
    nat = Image.open(os.path.join(REF, "uploads/anh1.jpg")).convert("RGB")
    nat_emb = ee.extract_embedding_single(os.path.join(REF, "uploads/anh1.jpg"), model, transform, "cpu")
    nat_tensor = transform(nat).numpy()

    # gallery with planted matches + distractors; reference recognize_with_db (dict db, stable sort)
    G = planted_gallery(batch, 1000, seed=1)
    names = [f"id_{i:04d}" for i in range(len(G))]
    eng = re_.RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.5)
    eng.db = {n: G[i] for i, n in enumerate(names)}
    top_names, top_scores, best = [], [], []
    for e in single:
        name, score, top5 = eng.recognize_with_db(e)
        best.append(name)
        top_names.append([names.index(t[0]) for t in top5])
        top_scores.append([t[1] for t in top5])
    # exact ties: duplicate rows keep insertion order (lowest index first)
    eng.db = {"dup_a": G[3], "dup_b": G[3].copy(), "other": G[5]}
    tie = eng.recognize_with_db(single[3])
    # cosine_similarity branches (norm ~1 -> dot; else dot/(|a||b|); zero -> 0.0)
    a, b = single[0], G[7] * 3.0
    cos_cases = np.array([re_.cosine_similarity(a, G[7]), re_.cosine_similarity(a, b),
                          re_.cosine_similarity(a, np.zeros(512, np.float32))], np.float32)
    # notebook batched match: np.dot + argmax (evaluate_arcface_kaggle.ipynb cell 15)
    argmax = np.argmax(np.dot(batch, G.T), axis=1)
    # Unknown threshold path
    eng.db = {n: G[i] for i, n in enumerate(names)}
    eng.set_threshold(0.999)
    unk = eng.recognize_with_db(single[0])

    np.savez_compressed(
        out,
        seed=np.array(1234), num_classes=np.array(num_classes),
        probes=probes, emb_single=single.astype(np.float32), emb_batch=batch.astype(np.float32),
        emb_raw=raw.numpy().astype(np.float32),
        natural_tensor=nat_tensor.astype(np.float32), natural_emb=np.asarray(nat_emb, np.float32),
        gallery_seed=np.array(1), gallery_rows=np.array(len(G)), gallery_sum=np.float64(G.astype(np.float64).sum()),
        top5_idx=np.array(top_names, np.int64),
        top5_scores=np.array(top_scores, np.float32), best_name=np.array(best),
        tie_name=np.array(tie[0]), tie_top=np.array([t[0] for t in tie[2]]),
        cos_cases=cos_cases, argmax=argmax.astype(np.int64),
        unknown_name=np.array(unk[0]), unknown_score=np.float32(unk[1]),
    )
    print(f"wrote {out}: strict load {missing}, emb norms {np.linalg.norm(single, axis=1).round(6)}")
    print("top-1:", best, "argmax:", argmax.tolist(), "tie:", tie[0], [t[0] for t in tie[2]])


if __name__ == "__main__":
    main()
