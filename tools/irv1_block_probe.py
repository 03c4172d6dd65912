import ctypes, sys, torch
sys.path.insert(0, '.')
from facerecognition_amd import _native as N
from facerecognition_amd.model import FRModel
from facerecognition_amd.synthetic import synthetic_crops
m = FRModel.synthetic("irv1_facenet", max_batch=256)
for B in (1, 4, 16, 32, 64, 128, 256):
    x = torch.from_numpy(synthetic_crops(B, 160, seed=1)).cuda()
    for _ in range(2):
        m.embed(x)
    torch.cuda.synchronize()
    buf = ctypes.create_string_buffer(1 << 20)
    N.check(N.lib().fr_debug_plan(m.handle, B, buf, len(buf)), "plan")
    toks = [l.split()[0] for l in buf.value.decode().splitlines() if l.strip()]
    print(B, {t: toks.count(t) for t in set(toks)}, flush=True)
