"""Bit-for-bit comparison of two libfrhip builds on the same synthetic model and crops.

    FR_LIBFRHIP=<lib A> python tools/lib_bitcheck.py dump a.npz
    FR_LIBFRHIP=<lib B> python tools/lib_bitcheck.py dump b.npz
    python tools/lib_bitcheck.py cmp a.npz b.npz

Write the .npz files outside gpurun_out/ (they are tens of MB; gpurun copies back at most 64 MiB).
Used when a kernel is restructured without changing any product's summation order (e.g. the layer3
stage's 13-fragment layout): the embeddings and the kept stage intermediates must be identical."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def dump(path, arch="iresnet100", B=6):
    import ctypes
    import torch
    from facerecognition_amd import _native as N
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    L = N.lib()
    out = {}
    for stage in (2, 1):
        m = FRModel.synthetic(arch)
        m.set_option(N.FR_OPT_STAGE, stage)
        m.set_option(N.FR_OPT_KEEP_INTERMEDIATES, 1)
        x = torch.from_numpy(synthetic_crops(B, 112, seed=11))
        out[f"emb_stage{stage}"] = m.embed(x).cpu().numpy()
        for t in range(L.fr_debug_tensor_count(m.handle)):
            name = L.fr_debug_tensor_name(m.handle, t).decode()
            if not name.startswith("layer3"):
                continue
            H, W, C = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            N.check(L.fr_debug_tensor_shape(m.handle, t, ctypes.byref(H), ctypes.byref(W), ctypes.byref(C)))
            buf = torch.empty((B, H.value, W.value, C.value), dtype=torch.bfloat16, device="cuda")
            N.check(L.fr_debug_copy_tensor(m.handle, t, B, buf.data_ptr(), N.stream_ptr()))
            torch.cuda.synchronize()
            out[f"s{stage}_{name}"] = buf.view(torch.int16).cpu().numpy()
        m.close()
    np.savez(path, **out)
    print(f"dumped {len(out)} arrays to {path}")


def cmp(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = [k for k in A.files if k not in Bz.files or not np.array_equal(A[k], Bz[k])]
    print(f"{len(A.files) - len(bad)}/{len(A.files)} identical" + (f"; differ: {bad[:10]}" if bad else ""))
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
