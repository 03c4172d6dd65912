"""In-launch split-K reduction (conv_igemm.hip): the last workgroup of each tile sums the tile's partials in split
order and runs the split-K epilogue's arithmetic, replacing the second (splitk_epilogue_kernel) launch.  Same
bits either way: a model forward with FR_OPT_SPLITK_INLAUNCH on equals the one with it off, at the small
batches whose plans take split-K convs (the reference's online path, recognition_engine.py:328-381)."""
import ctypes

import numpy as np
import pytest
import torch

from facerecognition_amd import _native as N

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("arch,B", [("iresnet100", 1), ("iresnet100", 3), ("resnet50_arcface", 2)])
def test_splitk_inlaunch_equals_epilogue_launch(gpu, arch, B):
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic(arch)
    assert m.get_option(N.FR_OPT_SPLITK_INLAUNCH) == 1
    x = torch.from_numpy(synthetic_crops(B, m.input_size, seed=5 + B))
    a = m.embed(x).cpu().numpy()  # tuning forward (kernel choice per conv measured at this batch size)
    a = m.embed(x).cpu().numpy()
    buf = ctypes.create_string_buffer(1 << 16)
    N.check(N.lib().fr_debug_plan(m.handle, B, buf, len(buf)), "fr_debug_plan")
    splits = [l for l in buf.value.decode().splitlines()
              if l.startswith("conv ") and abs(int(l.split()[6])) > 1 and int(l.split()[5]) != N.FR_TILE_SMALL]
    m.set_option(N.FR_OPT_SPLITK_INLAUNCH, 0)
    b = m.embed(x).cpu().numpy()
    m.set_option(N.FR_OPT_SPLITK_INLAUNCH, 1)
    c = m.embed(x).cpu().numpy()
    m.close()
    assert np.array_equal(a, b) and np.array_equal(a, c), f"max |diff| {np.abs(a - b).max():.3g}"
    if not splits:
        pytest.skip(f"{arch} bs={B}: the measured plan took no igemm split-K conv")
    print(f"{arch} bs={B}: {len(splits)} split-K convs, {sum(int(l.split()[6]) < 0 for l in splits)} reduced in-launch")


@pytest.mark.parametrize("inlaunch", [0, 1])
def test_graph_replay_after_other_batch_sizes(gpu, inlaunch):
    """A bs = 1 forward captured as a hipGraph and replayed after forwards at other batch sizes (tuning passes,
    their own captures) returns the embeddings it returned before (tests/test_gpu_host_api.py's call order:
    recognize_batch, then recognize).  In-launch split-K failed exactly this (1-cos 0.15, deterministic) while its
    partial slabs went through plain stores and loads behind the agent-scope release / acquire pair; with sc1
    stores and loads it passes."""
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    m = FRModel.synthetic("resnet50_arcface")
    m.set_option(N.FR_OPT_SPLITK_INLAUNCH, inlaunch)
    x = torch.from_numpy(synthetic_crops(9, m.input_size, seed=21)).to(gpu)
    x1 = x[:1].clone()
    out = torch.empty((1, 512), dtype=torch.float32, device=gpu)
    first = []
    for _ in range(4):  # tuning forward, first sighting, capture + replay, replay
        m.embed(x1, out=out)
        first.append(out.cpu().numpy().copy())
    m.embed(x[:8])
    m.embed(x)
    m.embed(x[:8])
    later = []
    for _ in range(3):
        m.embed(x1, out=out)
        later.append(out.cpu().numpy().copy())
    m.close()
    for e in first[1:] + later:
        assert np.array_equal(e, first[0]), f"max |diff| {np.abs(e - first[0]).max():.3g}"
