"""CPU oracle for the face-embedding + gallery-match path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / the timed CPU baseline.  The product path
(``facerecognition_amd``) never imports it and fails loudly when libfrhip.so is missing.

Contents (each function cites the reference file:line it restates):
  models.py — PyTorch fp32 CPU restatements of the three backbones:
      ResNet-50 ``ArcFaceModel`` (parity PINNED: tests/golden/arcface_r50_golden.npz was produced
      by importing the reference's own models/arcface/arcface_model.py + inference/*.py in the
      survey container, see tools/gen_golden.py);
      IResNet100 and InceptionResnetV1 — no reference code ships for them (README-only /
      external facenet-pytorch), so their parity is UNPINNED beyond self-consistency.
  match.py  — numpy restatements of cosine_similarity, recognize_with_db, the notebook's
      batched np.dot + argmax/argsort, FAISS IndexFlatIP search, prototypes/folder means.
"""
