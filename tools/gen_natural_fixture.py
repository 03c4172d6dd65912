"""Writes tests/golden/anh1_u8.npz: the reference's one natural image, uploads/anh1.jpg (900x900 RGB),
decoded by PIL to u8 HWC.  Data only (the decoded pixels), so tests and the GPU box never need the
reference tree or a JPEG decoder of the same version.  Run in the survey container:
    python tools/gen_natural_fixture.py /root/reference/uploads/anh1.jpg"""
import os
import sys

import numpy as np
from PIL import Image

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/uploads/anh1.jpg"
u8 = np.asarray(Image.open(src).convert("RGB"), dtype=np.uint8)
out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "anh1_u8.npz")
np.savez_compressed(out, u8=u8)
print(out, u8.shape)
