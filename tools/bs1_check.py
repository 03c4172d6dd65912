#!/usr/bin/env python3
"""Small-batch consistency check: each model's bs = 1..4 embeddings against the same images inside a bs = 9 batch
(1 - cos per face; bf16-rounding level expected).  python tools/bs1_check.py [arch ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(archs):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    for arch in archs:
        m = FRModel.synthetic(arch)
        x = torch.from_numpy(synthetic_crops(9, m.input_size, seed=3))
        ref = m.embed(x).cpu().numpy()
        for B in (1, 2, 4):
            e = m.embed(x[:B]).cpu().numpy()
            e = m.embed(x[:B]).cpu().numpy()
            d = 1.0 - (e * ref[:B]).sum(1)
            print(f"{arch} B={B}: max 1-cos vs bs=9 {d.max():.3g}", flush=True)
        m.close()




def recognize_repro():
    """tests/test_gpu_host_api.py::test_recognize_batch_end_to_end, with the numpy scores of both embeddings."""
    from PIL import Image
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.recognition_engine import RecognitionEngine
    from facerecognition_amd.synthetic import planted_gallery
    from facerecognition_amd.weights import synth_state_dict
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gold = np.load(os.path.join(root, "tests/golden/arcface_r50_golden.npz"))
    sd = synth_state_dict("resnet50_arcface", seed=int(gold["seed"]), num_classes=int(gold["num_classes"]))
    r50 = FRModel("resnet50_arcface", sd, max_batch=64)
    G = planted_gallery(gold["emb_batch"], int(gold["gallery_rows"]), seed=int(gold["gallery_seed"]))
    db = {f"id_{i:04d}": G[i] for i in range(len(G))}
    eng = RecognitionEngine(model_path=None, use_face_detection=False, threshold=0.5, model=r50)
    eng.db = db
    imgs = [Image.fromarray(p) for p in gold["probes"]]
    res = eng.recognize_batch(imgs)
    single = eng.recognize(imgs[2])
    e1, e9 = single["embedding"], res[2]["embedding"]
    Gn = G / np.linalg.norm(G, axis=1, keepdims=True)
    print("cos(single, batch)", float(e1 @ e9 / np.linalg.norm(e1) / np.linalg.norm(e9)))
    print("conf single/batch", single["confidence"], res[2]["confidence"])
    print("numpy best single/batch", float((Gn @ e1).max()), float((Gn @ e9).max()))
    print("top single", single["top_k"][:3], "batch", res[2]["top_k"][:3])
    print("norms", float(np.linalg.norm(e1)), float(np.linalg.norm(e9)))


def host_api_repro():
    """tests/test_gpu_host_api.py's call order on one model (bs = 1 u8 x8, bs = 1 f32, bs = 8 raw, bs = 9, bs = 1)."""
    import torch
    from PIL import Image
    from facerecognition_amd.extract_embeddings import extract_embedding_single, get_transform
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.weights import synth_state_dict
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gold = np.load(os.path.join(root, "tests/golden/arcface_r50_golden.npz"))
    sd = synth_state_dict("resnet50_arcface", seed=int(gold["seed"]), num_classes=int(gold["num_classes"]))
    m = FRModel("resnet50_arcface", sd, max_batch=64)
    cd = lambda a, b: float(1 - (a * b).sum() / np.linalg.norm(a) / np.linalg.norm(b))
    t = get_transform()
    e = [extract_embedding_single(Image.fromarray(p), m, t) for p in gold["probes"]]
    print("single x8 max", max(cd(e[i], gold["emb_single"][i]) for i in range(8)))
    m.embed(torch.from_numpy(gold["natural_tensor"])[None])
    m(torch.from_numpy(gold["probes"]))
    x = torch.from_numpy(gold["probes"])
    m.embed(x)
    for r in range(4):
        e2 = extract_embedding_single(Image.fromarray(gold["probes"][2]), m, t)
        print("after: single[2]", r, cd(e2, gold["emb_single"][2]), flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["recognize"]:
        recognize_repro()
    elif sys.argv[1:] == ["host_api"]:
        host_api_repro()
    else:
        main(sys.argv[1:] or ["resnet50_arcface", "iresnet100", "irv1_facenet"])
