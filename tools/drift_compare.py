"""Per-stage relative error vs the fp32 oracle for two dtypes side by side (tests/test_gpu_layers.py's
stage_report):  python tools/drift_compare.py irv1_facenet bf16 f16"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_layers import stage_report  # noqa: E402

arch, d1, d2 = sys.argv[1], sys.argv[2], sys.argv[3]
a = {n: r for n, _, r in stage_report(arch, B=4, dtype=d1)}
b = {n: r for n, _, r in stage_report(arch, B=4, dtype=d2)}
for n in a:
    print(f"{n:34s} {d1} {a[n]:.3e}   {d2} {b.get(n, float('nan')):.3e}   ratio {a[n] / max(b.get(n, 1e-30), 1e-30):6.1f}")
