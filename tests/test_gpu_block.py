"""LDS-resident Inception-ResNet blocks (conv_block.hip): FaceNet IRV1's Block35 / Block17 / Block8 as one
launch each, against their member convs run one by one through fr_op_conv2d with conv_igemm tile 0 (no
split-K).  The block keeps every branch intermediate in LDS but rounds it to the plan's 16-bit type exactly
where the per-conv path stores it, runs each conv's 32-deep MFMA chain over k in order and applies the igemm
epilogue, so the block output must equal the per-conv chain bit for bit (reference block structure:
facenet_model.py:28-36 -> facenet-pytorch Block35 / Block17 / Block8)."""
import numpy as np
import pytest
import torch

from facerecognition_amd import _native as N
from tests.helpers import conv_op
from tests.test_gpu_stage import _named

pytestmark = pytest.mark.gpu


def _w(folded, name):
    """folded KRSC f32 weights -> conv_op's [Cout, Cin, kh, kw] f32, and the bias."""
    w = torch.from_numpy(folded[name + ".w"]).permute(0, 3, 1, 2).contiguous()
    return w, torch.from_numpy(folded[name + ".b"])


def _cat(folded, names):
    ws, bs = zip(*[_w(folded, n) for n in names])
    return torch.cat(ws, 0), torch.cat(bs, 0)


def _block35(x, f, p):
    w, b = _cat(f, [p + "branch1.0", p + "branch2.0", p + "branch0"])
    t = conv_op(x, w, bias=b, act=1, tile=0)                       # [t1 | t2 | b0]
    w, b = _w(f, p + "branch1.1")
    b1 = conv_op(t, w, bias=b, act=1, pad=(1, 1), x_off=0, cin=32, tile=0)
    w, b = _w(f, p + "branch2.1")
    t2 = conv_op(t, w, bias=b, act=1, pad=(1, 1), x_off=32, cin=32, tile=0)
    w, b = _w(f, p + "branch2.2")
    b2 = conv_op(t2, w, bias=b, act=1, pad=(1, 1), tile=0)
    cat = torch.cat([t[..., 64:96], b1, b2], -1).contiguous()
    w, b = _w(f, p + "conv2d")
    return conv_op(cat, w, bias=b, res=x, act=1, tile=0)


def _block17_8(x, f, p, k, act):
    w, b = _cat(f, [p + "branch1.0", p + "branch0"])
    t = conv_op(x, w, bias=b, act=1, tile=0)                       # [t1 | b0]
    c = w.shape[0] // 2
    w, b = _w(f, p + "branch1.1")                                  # 1 x k
    u = conv_op(t, w, bias=b, act=1, pad=(0, k // 2), x_off=0, cin=c, tile=0)
    w, b = _w(f, p + "branch1.2")                                  # k x 1
    b1 = conv_op(u, w, bias=b, act=1, pad=(k // 2, 0), tile=0)
    cat = torch.cat([t[..., c:], b1], -1).contiguous()
    w, b = _w(f, p + "conv2d")
    return conv_op(cat, w, bias=b, res=x, act=act, tile=0)


@pytest.mark.parametrize("B", [1, 9])
def test_irv1_blocks_equal_member_convs(gpu, B):
    from facerecognition_amd import weights as Wt
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops
    arch = "irv1_facenet"
    f = Wt.fold_state_dict(arch, Wt.synth_state_dict(arch, seed=1234))
    m = FRModel.synthetic(arch, seed=1234)
    assert m.get_option(N.FR_OPT_STAGE) == 1  # the blocks make the stage option apply to IRV1
    m.set_option(N.FR_OPT_STAGE, 2)          # blocks always on
    x = torch.from_numpy(synthetic_crops(B, 160, seed=11))
    e_blk = m.embed(x).cpu().numpy()
    import ctypes
    buf = ctypes.create_string_buffer(1 << 16)
    N.check(N.lib().fr_debug_plan(m.handle, B, buf, len(buf)), "fr_debug_plan")
    plan = buf.value.decode().splitlines()
    assert sum(l.startswith("block ") for l in plan) == 21, "the 21 blocks did not all run as conv_block launches"
    M = "model."
    pairs = [("conv2d_4b", "repeat_1.0"), ("repeat_1.3", "repeat_1.4"), ("mixed_6a", "repeat_2.0"),
             ("repeat_2.8", "repeat_2.9"), ("mixed_7a", "repeat_3.0"), ("repeat_3.4", "block8")]
    t = _named(m, B, {M + a for a, _ in pairs} | {M + b for _, b in pairs})
    for a, b in pairs:
        xin = t[M + a].to(torch.bfloat16).cuda()
        p = M + b + "."
        if b.startswith("repeat_1"):
            ref = _block35(xin, f, p)
        elif b.startswith("repeat_2"):
            ref = _block17_8(xin, f, p, 7, 1)
        else:
            ref = _block17_8(xin, f, p, 3, 0 if b == "block8" else 1)
        got = t[M + b]
        assert torch.equal(got, ref.float().cpu()), \
            f"{b}: block vs member convs max |diff| {(got - ref.float().cpu()).abs().max().item():.3g}"
    # the per-conv path of the same plan: same embeddings up to its kernels' summation order
    m.set_option(N.FR_OPT_STAGE, 0)
    e_conv = m.embed(x).cpu().numpy()
    m.close()
    cos = np.sum(e_blk * e_conv, axis=1)
    assert np.all(1 - cos <= 3e-4), f"block vs per-conv embeddings: 1-cos = {1 - cos}"
