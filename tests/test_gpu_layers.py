"""Per-stage drift: every named intermediate tensor of the native plan vs the output of the
oracle module with the same name (SURVEY.md §7 'Hard parts': measure bf16 drift per stage).

A wiring bug shows up as an O(1) relative error at the first wrong stage; bf16 rounding
drift stays at the few-percent level through 100+ layers."""
import ctypes

import numpy as np
import pytest
import torch

from facerecognition_amd import _native as N

pytestmark = pytest.mark.gpu

REL_TOL = 0.08  # per-stage relative L2 error bound (bf16 storage of every activation)


def stage_report(arch, B=2, seed=0, dtype=None):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.weights import INPUT_SIZE, synth_state_dict
    from oracle import models as M

    from facerecognition_amd.synthetic import synthetic_crops
    u8 = synthetic_crops(B, INPUT_SIZE[arch], seed=seed)
    sd = synth_state_dict(arch)
    m = FRModel(arch, sd, dtype=dtype)
    m.set_option(N.FR_OPT_KEEP_INTERMEDIATES, 1)  # the layer3 stage kernel materialises its blocks too
    m.embed(torch.from_numpy(u8))
    torch.cuda.synchronize()
    L = N.lib()
    ours = {}
    for t in range(L.fr_debug_tensor_count(m.handle)):
        name = L.fr_debug_tensor_name(m.handle, t).decode()
        if not name:
            continue
        H, W, C = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        N.check(L.fr_debug_tensor_shape(m.handle, t, ctypes.byref(H), ctypes.byref(W), ctypes.byref(C)))
        # storage dtype per tensor (a bf16 IRV1 plan keeps its stem in f16)
        dt = torch.float16 if L.fr_debug_tensor_dtype(m.handle, t) == N.FR_DTYPE_F16 else torch.bfloat16
        buf = torch.empty((B, H.value, W.value, C.value), dtype=dt, device="cuda")
        N.check(L.fr_debug_copy_tensor(m.handle, t, B, buf.data_ptr(), N.stream_ptr()))
        torch.cuda.synchronize()
        ours[name] = buf.float().cpu()
    ref = {}
    om = M.build_model(arch, sd)
    hooks = []
    for name in ours:
        mod = om.get_submodule(name)
        hooks.append(mod.register_forward_hook(
            lambda _m, _i, o, name=name: ref.__setitem__(name, o.detach().clone())))
    M.embed(om, arch, u8)
    for h in hooks:
        h.remove()
    rows = []
    for name, got in ours.items():
        r = ref[name]
        r = r.permute(0, 2, 3, 1) if r.dim() == 4 else r.view(got.shape)
        rel = ((got - r).norm() / (r.norm() + 1e-12)).item()
        rows.append((name, tuple(got.shape), rel))
    m.close()
    return rows


@pytest.mark.parametrize("arch", ["resnet50_arcface", "iresnet100", "irv1_facenet"])
def test_stage_drift(gpu, arch):
    rows = stage_report(arch)
    worst = max(r[2] for r in rows)
    print(f"\n{arch}: {len(rows)} stages, worst rel err {worst:.3e}")
    for name, shp, rel in rows:
        print(f"  {name:28s} {str(shp):22s} {rel:.3e}")
    bad = [(n, r) for n, _, r in rows if r > REL_TOL]
    assert not bad, f"first stage over tolerance: {bad[0]}"
