"""Kernel-level parity: every libfrhip op vs a torch fp32 / numpy reference of the same op.

Tolerances: conv/linear operands are bf16-exact in both paths and both accumulate in f32,
so the only differences are summation order and the final bf16 rounding of the output
(relative 2^-8): |got - ref| <= 1e-2 * (|ref| + max|ref|/8).  Pool / preprocess are exact.
The match kernel is exact f32 (fmaf chain): scores within 1e-5, indices identical wherever the
reference's top-k gap exceeds 1e-5, and identical on constructed ties.
"""
import ctypes

import numpy as np
import pytest
import torch

from facerecognition_amd import _native as N
from tests.helpers import TORCH_DT, bf16_round, conv_op, conv_ref, q16

pytestmark = pytest.mark.gpu


def _close(got, ref, tol=1e-2):
    got = got.float().cpu()
    ref = ref.float().cpu()
    scale = ref.abs().max().item() + 1e-6
    err = (got - ref).abs()
    bound = tol * (ref.abs() + scale / 8)
    bad = (err > bound).sum().item()
    assert bad == 0, f"{bad} / {err.numel()} elements out of tolerance; max err {err.max().item():.4g} (scale {scale:.4g})"


CONV_CASES = [
    # B, H, W, Cin, Cout, kh, kw, stride, pad
    (2, 14, 14, 256, 256, 3, 3, (1, 1), (1, 1)),   # IResNet100 layer3 conv
    (2, 28, 28, 128, 128, 3, 3, (2, 2), (1, 1)),   # stride-2 block conv
    (2, 56, 56, 64, 64, 3, 3, (1, 1), (1, 1)),     # layer1 (BN=64 tile)
    (3, 7, 7, 512, 512, 3, 3, (1, 1), (1, 1)),     # layer4
    (2, 16, 16, 64, 256, 1, 1, (1, 1), (0, 0)),    # bottleneck expand
    (2, 16, 16, 256, 128, 1, 1, (2, 2), (0, 0)),   # 1x1 stride-2 downsample
    (2, 30, 30, 8, 64, 7, 7, (2, 2), (3, 3)),      # ResNet-50 stem (Cin padded to 8)
    (2, 20, 20, 8, 64, 3, 3, (1, 1), (1, 1)),      # IResNet stem
    (2, 21, 21, 8, 32, 3, 3, (2, 2), (0, 0)),      # IRV1 conv2d_1a
    (2, 19, 19, 80, 192, 3, 3, (1, 1), (0, 0)),    # IRV1 conv2d_4a (Cin=80, K not /64)
    (2, 8, 8, 128, 128, 1, 7, (1, 1), (0, 3)),     # Block17 1x7
    (2, 8, 8, 128, 128, 7, 1, (1, 1), (3, 0)),     # Block17 7x1
    (2, 5, 5, 192, 192, 1, 3, (1, 1), (0, 1)),     # Block8 1x3
    (2, 9, 9, 32, 32, 3, 3, (1, 1), (1, 1)),       # Block35 3x3 (Cin=32)
    (1, 3, 3, 1792, 384, 1, 1, (1, 1), (0, 0)),    # Block8 fused 1x1 (tiny M)
]


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_parity(gpu, case, dtype):
    B, H, W, Cin, Cout, kh, kw, stride, pad = case
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    x = torch.randn(B, H, W, Cin, generator=g).to(TORCH_DT[dtype]).to(gpu)
    w = torch.randn(Cout, Cin, kh, kw, generator=g) / np.sqrt(Cin * kh * kw)
    bias = torch.randn(Cout, generator=g) * 0.1
    y = conv_op(x, w, stride=stride, pad=pad, bias=bias, act=1, dtype=dtype)
    ref = conv_ref(x, w, stride=stride, pad=pad, bias=bias, act=1, dtype=dtype)
    _close(y, ref, tol=1e-2 if dtype == "bf16" else 2e-3)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 8, 9])
@pytest.mark.parametrize("case", [(2, 14, 14, 256, 256, 3, 3, (1, 1), (1, 1)), (2, 19, 19, 80, 192, 3, 3, (1, 1), (0, 0)),
                                  (3, 9, 9, 64, 64, 1, 1, (2, 2), (0, 0))])
def test_conv_every_tile(gpu, case, tile):
    B, H, W, Cin, Cout, kh, kw, stride, pad = case
    g = torch.Generator().manual_seed(tile)
    x = torch.randn(B, H, W, Cin, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(Cout, Cin, kh, kw, generator=g) / np.sqrt(Cin * kh * kw)
    y = conv_op(x, w, stride=stride, pad=pad, act=1, tile=tile)
    _close(y, conv_ref(x, w, stride=stride, pad=pad, act=1))


BAND_CASES = [(2, 14, 14, 256, 256), (2, 28, 28, 128, 128), (2, 56, 56, 64, 64), (1, 112, 112, 64, 64),
              (2, 14, 14, 128, 256), (2, 28, 28, 64, 128), (2, 28, 28, 128, 256), (2, 28, 28, 64, 64),
              (3, 14, 14, 512, 256), (1, 14, 14, 256, 512), (2, 14, 14, 192, 256), (1, 28, 28, 256, 128)]


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("case", BAND_CASES)
def test_conv_band(gpu, case, dtype):
    """Row-band direct 3x3/s1/p1 kernel (forced) with the IResNet epilogue: bias + residual +
    PReLU + second affine output."""
    B, H, W, Cin, Cout = case
    g = torch.Generator().manual_seed(Cin + Cout + H)
    x = torch.randn(B, H, W, Cin, generator=g).to(TORCH_DT[dtype]).to(gpu)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / np.sqrt(Cin * 9)
    bias = torch.randn(Cout, generator=g) * 0.1
    slope = torch.rand(Cout, generator=g) * 0.5
    res = torch.randn(B, H, W, Cout, generator=g).to(TORCH_DT[dtype]).to(gpu)
    s = torch.rand(Cout, generator=g) + 0.5
    t = torch.randn(Cout, generator=g) * 0.1
    y2 = torch.zeros(B, H, W, Cout, dtype=TORCH_DT[dtype], device=gpu)
    y = conv_op(x, w, pad=(1, 1), bias=bias, act=2, slope=slope, res=res, y2=y2, aff_s=s, aff_b=t, dtype=dtype,
                tile=N.FR_TILE_BAND)
    ref = conv_ref(x, w, pad=(1, 1), bias=bias, act=2, slope=slope, res=res, dtype=dtype)
    tol = 1e-2 if dtype == "bf16" else 2e-3
    _close(y, ref, tol=tol)
    _close(y2, y.float().cpu() * s + t, tol=tol)


@pytest.mark.parametrize("dtype", ["bf16"])  # (f16 nets have no 28x28x128 convs: the kernel is bf16-only)
@pytest.mark.parametrize("B", [1, 3])
def test_conv_img28(gpu, B, dtype):
    """Image-per-workgroup layer2 kernel (conv_img.hip, forced): 3x3/s1/p1 28x28 128->128 with the
    IResNet conv2 epilogue (bias + residual) and the conv1 one (PReLU)."""
    g = torch.Generator().manual_seed(28 + B)
    x = torch.randn(B, 28, 28, 128, generator=g).to(TORCH_DT[dtype]).to(gpu)
    w = torch.randn(128, 128, 3, 3, generator=g) / np.sqrt(128 * 9)
    bias = torch.randn(128, generator=g) * 0.1
    slope = torch.rand(128, generator=g) * 0.5
    res = torch.randn(B, 28, 28, 128, generator=g).to(TORCH_DT[dtype]).to(gpu)
    tol = 1e-2 if dtype == "bf16" else 2e-3
    y = conv_op(x, w, pad=(1, 1), bias=bias, res=res, dtype=dtype, tile=N.FR_TILE_IMG28)
    _close(y, conv_ref(x, w, pad=(1, 1), bias=bias, res=res, dtype=dtype), tol=tol)
    y = conv_op(x, w, pad=(1, 1), bias=bias, act=2, slope=slope, dtype=dtype, tile=N.FR_TILE_IMG28)
    _close(y, conv_ref(x, w, pad=(1, 1), bias=bias, act=2, slope=slope, dtype=dtype), tol=tol)


@pytest.mark.parametrize("B", [1, 3])
def test_conv_img56(gpu, B):
    """Layer-1 instance of the band kernel (conv_img.hip, 56x56 64->64, 4-row bands, forced)."""
    g = torch.Generator().manual_seed(56 + B)
    x = torch.randn(B, 56, 56, 64, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(64, 64, 3, 3, generator=g) / np.sqrt(64 * 9)
    bias = torch.randn(64, generator=g) * 0.1
    slope = torch.rand(64, generator=g) * 0.5
    res = torch.randn(B, 56, 56, 64, generator=g).to(torch.bfloat16).to(gpu)
    y = conv_op(x, w, pad=(1, 1), bias=bias, res=res, tile=N.FR_TILE_IMG56)
    _close(y, conv_ref(x, w, pad=(1, 1), bias=bias, res=res))
    y = conv_op(x, w, pad=(1, 1), bias=bias, act=2, slope=slope, tile=N.FR_TILE_IMG56)
    _close(y, conv_ref(x, w, pad=(1, 1), bias=bias, act=2, slope=slope))


ROWS_CASES = [(1, 56, 56, 64), (3, 56, 56, 64), (1, 112, 112, 64), (2, 56, 56, 128), (2, 112, 56, 64),
              (5, 56, 112, 128)]


@pytest.mark.parametrize("case", ROWS_CASES)
def test_conv_rows(gpu, case):
    """Persistent weight-resident 64-input-channel kernel (conv_rows.hip, forced): the IResNet conv2
    epilogue (bias + residual) and the conv1 one (PReLU), Cout 64 and 128 (two n-groups), 56- and
    112-wide images (column halves), non-square images, batches whose unit count does not divide the
    grid."""
    B, H, W, Cout = case
    g = torch.Generator().manual_seed(H + W + Cout + B)
    x = torch.randn(B, H, W, 64, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(Cout, 64, 3, 3, generator=g) / np.sqrt(64 * 9)
    bias = torch.randn(Cout, generator=g) * 0.1
    slope = torch.rand(Cout, generator=g) * 0.5
    res = torch.randn(B, H, W, Cout, generator=g).to(torch.bfloat16).to(gpu)
    y = conv_op(x, w, pad=(1, 1), bias=bias, res=res, tile=N.FR_TILE_ROWS)
    _close(y, conv_ref(x, w, pad=(1, 1), bias=bias, res=res))
    y = conv_op(x, w, pad=(1, 1), bias=bias, act=2, slope=slope, tile=N.FR_TILE_ROWS)
    _close(y, conv_ref(x, w, pad=(1, 1), bias=bias, act=2, slope=slope))
    # same bits as the implicit GEMM up to f32 summation order: compare against tile 0 tightly
    y0 = conv_op(x, w, pad=(1, 1), bias=bias, act=2, slope=slope, tile=0)
    _close(y, y0.float().cpu(), tol=1e-2)


WRING_CASES = [  # (B, H, W, Cin, Cout, stride): layer4 (two 7x7 images per block, M not a multiple of
    # 112 at B = 3), layer3.0.conv1, the layer4.0 stride-2 conv, a 28x28 stride-2 one
    (3, 7, 7, 512, 512, 1), (1, 28, 28, 128, 256, 1), (2, 14, 14, 256, 512, 2), (2, 28, 28, 128, 256, 2),
    (2, 28, 28, 128, 128, 1), (1, 56, 56, 64, 128, 2)]  # 128-channel blocks (4 waves); Kpad % 128 == 64


@pytest.mark.parametrize("case", WRING_CASES)
def test_conv_wring(gpu, case):
    """Register-weight-ring implicit GEMM (conv_wring.hip, forced): bias + residual, PReLU and the
    border-class bias epilogues; it sums K in the igemm's order, so it must equal tile 0 bit for bit."""
    B, H, W, Cin, Cout, st = case
    g = torch.Generator().manual_seed(B + H + Cin + Cout + st)
    x = torch.randn(B, H, W, Cin, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / np.sqrt(Cin * 9)
    bias = torch.randn(Cout, generator=g) * 0.1
    slope = torch.rand(Cout, generator=g) * 0.5
    Ho = (H + 2 - 3) // st + 1
    res = torch.randn(B, Ho, Ho, Cout, generator=g).to(torch.bfloat16).to(gpu)
    kw = dict(stride=(st, st), pad=(1, 1))
    y = conv_op(x, w, bias=bias, res=res, tile=N.FR_TILE_WRING, **kw)
    _close(y, conv_ref(x, w, bias=bias, res=res, **kw))
    assert torch.equal(y, conv_op(x, w, bias=bias, res=res, tile=0, **kw))
    b9 = torch.randn(9, Cout, generator=g) * 0.1
    y = conv_op(x, w, act=2, slope=slope, bias9=b9, tile=N.FR_TILE_WRING, **kw)
    assert torch.equal(y, conv_op(x, w, act=2, slope=slope, bias9=b9, tile=0, **kw))
    with pytest.raises(RuntimeError, match="wring"):  # Cout % 128 != 0: refused, no silent fallback
        conv_op(x, torch.randn(64, Cin, 3, 3, generator=g), pad=(1, 1), tile=N.FR_TILE_WRING)


TILE64_CASES = [  # (B, H, W, Cin, Cout, kh, kw, pad): IRV1 Block8 / mixed_7a shapes (M = 9 B), a ragged M, Cin % 64 != 0
    (4, 3, 3, 1792, 384, 1, 1, (0, 0)), (4, 3, 3, 192, 192, 1, 3, (0, 1)), (4, 3, 3, 384, 1792, 1, 1, (0, 0)),
    (3, 8, 8, 256, 256, 3, 3, (1, 1)), (2, 5, 7, 96, 64, 3, 3, (1, 1))]


@pytest.mark.parametrize("tile", ["FR_TILE_64x64_S3", "FR_TILE_64x64", "FR_TILE_32x64_S3"])
@pytest.mark.parametrize("case", TILE64_CASES)
def test_conv_tile64(gpu, case, tile):
    """The 64 x 64 implicit-GEMM tiles (round 6, autotuner candidates for small-M convs): they sum K in tile 0's
    order, so they must equal it bit for bit (bias + residual, bias + ReLU)."""
    B, H, W, Cin, Cout, kh, kw, pd = case
    g = torch.Generator().manual_seed(B + H + Cin + Cout + kh)
    x = torch.randn(B, H, W, Cin, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(Cout, Cin, kh, kw, generator=g) / np.sqrt(Cin * kh * kw)
    bias = torch.randn(Cout, generator=g) * 0.1
    res = torch.randn(B, H, W, Cout, generator=g).to(torch.bfloat16).to(gpu)
    t = getattr(N, tile)
    y = conv_op(x, w, pad=pd, bias=bias, res=res, tile=t)
    _close(y, conv_ref(x, w, pad=pd, bias=bias, res=res))
    assert torch.equal(y, conv_op(x, w, pad=pd, bias=bias, res=res, tile=0))
    assert torch.equal(conv_op(x, w, pad=pd, bias=bias, act=1, tile=t), conv_op(x, w, pad=pd, bias=bias, act=1, tile=0))


DIRECT_CASES = [
    # B, H, W, Cin, Cout, kh, kw, stride, pad, act   (FaceNet IRV1 shapes, smaller images)
    (2, 41, 41, 8, 32, 3, 3, (2, 2), (0, 0), 1),      # conv2d_1a (Cin padded to 8, K = 72)
    (2, 23, 23, 32, 32, 3, 3, (1, 1), (0, 0), 1),     # conv2d_2a (valid)
    (3, 40, 40, 32, 64, 3, 3, (1, 1), (1, 1), 1),     # conv2d_2b (several units per image)
    (2, 17, 17, 32, 32, 3, 3, (1, 1), (1, 1), 0),     # Block35 3x3
    (2, 17, 17, 256, 96, 1, 1, (1, 1), (0, 0), 2),    # Block35 fused 1x1 256 -> 3 x 32 (PReLU path)
    (2, 17, 17, 96, 256, 1, 1, (1, 1), (0, 0), 0),    # Block35 up 1x1 (K = 96)
    (2, 8, 8, 256, 896, 1, 1, (1, 1), (0, 0), 1),     # Block17 up 1x1 (14 channel groups)
    (1, 3, 3, 384, 1792, 1, 1, (1, 1), (0, 0), 0),    # Block8 up 1x1 (K = 384, the register limit)
]


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("case", DIRECT_CASES)
def test_conv_direct(gpu, case, dtype):
    """Persistent small-K direct conv (conv_direct.hip, forced): bias + ReLU / PReLU / none; it sums K in
    the igemm's 32-deep MFMA chunks and applies the igemm's epilogue arithmetic, so it must equal tile 0
    bit for bit (the autotuner times it beside the igemm tiles)."""
    B, H, W, Cin, Cout, kh, kw, st, pd, act = case
    g = torch.Generator().manual_seed(B + H + Cin + Cout + kh)
    x = torch.randn(B, H, W, Cin, generator=g).to(TORCH_DT[dtype]).to(gpu)
    w = torch.randn(Cout, Cin, kh, kw, generator=g) / np.sqrt(Cin * kh * kw)
    bias = torch.randn(Cout, generator=g) * 0.1
    slope = torch.rand(Cout, generator=g) * 0.5 if act == 2 else None
    kw_ = dict(stride=st, pad=pd, bias=bias, act=act, slope=slope, dtype=dtype)
    y = conv_op(x, w, tile=N.FR_TILE_DIRECT, **kw_)
    _close(y, conv_ref(x, w, stride=st, pad=pd, bias=bias, act=act, slope=slope, dtype=dtype))
    assert torch.equal(y, conv_op(x, w, tile=0, **kw_))


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("case", [
    # B, H, W, Cin, Cout, act   (1x1 / stride 1: operand B straight from global memory; + residual)
    (2, 17, 17, 96, 256, 1),    # Block35 up: x + conv(cat), ReLU (the 0.17 scale folded into the weights)
    (2, 8, 8, 256, 896, 1),     # Block17 up
    (3, 3, 3, 384, 1792, 0),    # Block8 up (K = 384, no activation on the last block)
    (2, 38, 38, 64, 96, 2),     # conv2d_3b-like (K = 64, Cout % 64 != 0)
])
def test_conv_direct_1x1_residual(gpu, case, dtype):
    """conv_direct's 1x1 kernel (operand B from global memory, two units in registers): bias + residual +
    activation; equal to igemm tile 0 bit for bit."""
    B, H, W, Cin, Cout, act = case
    g = torch.Generator().manual_seed(H + Cin + Cout)
    x = torch.randn(B, H, W, Cin, generator=g).to(TORCH_DT[dtype]).to(gpu)
    w = torch.randn(Cout, Cin, 1, 1, generator=g) / np.sqrt(Cin)
    bias = torch.randn(Cout, generator=g) * 0.1
    res = torch.randn(B, H, W, Cout, generator=g).to(TORCH_DT[dtype]).to(gpu)
    slope = torch.rand(Cout, generator=g) * 0.5 if act == 2 else None
    kw_ = dict(bias=bias, res=res, act=act, slope=slope, dtype=dtype)
    y = conv_op(x, w, tile=N.FR_TILE_DIRECT, **kw_)
    _close(y, conv_ref(x, w, bias=bias, res=res, act=act, slope=slope, dtype=dtype))
    assert torch.equal(y, conv_op(x, w, tile=0, **kw_))


def test_conv_direct_channel_slices_and_applicability(gpu):
    """Input / output channel slices (IRV1 concatenations: x_off / Cx, y_off / Cy); shapes past the register
    limit are refused (fail loudly, no silent fallback)."""
    g = torch.Generator().manual_seed(77)
    x = torch.randn(2, 17, 17, 320, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(32, 32, 3, 3, generator=g) / 17
    out = torch.randn(2, 17, 17, 128, generator=g).to(torch.bfloat16).to(gpu)
    before = out.clone()
    conv_op(x, w, pad=(1, 1), x_off=96, cin=32, act=1, y=out, y_off=64, tile=N.FR_TILE_DIRECT)
    _close(out[..., 64:96], conv_ref(x, w, pad=(1, 1), x_off=96, cin=32, act=1))
    ref = out.clone()
    out.copy_(before)
    conv_op(x, w, pad=(1, 1), x_off=96, cin=32, act=1, y=out, y_off=64, tile=0)
    assert torch.equal(out, ref)
    assert torch.equal(ref[..., :64], before[..., :64]) and torch.equal(ref[..., 96:], before[..., 96:])
    with pytest.raises(RuntimeError, match="direct"):  # K = 3 * 3 * 64 = 576 > 384
        conv_op(x[..., :64].contiguous(), torch.randn(64, 64, 3, 3, generator=g), pad=(1, 1), tile=N.FR_TILE_DIRECT)


def test_conv_img28_channel_slices_and_applicability(gpu):
    """img28 reads channels [128:256) of a 256-ch buffer and writes [64:192) of another; other shapes
    are refused (fail loudly, no silent fallback)."""
    g = torch.Generator().manual_seed(31)
    x = torch.randn(2, 28, 28, 256, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(128, 128, 3, 3, generator=g) / 34
    out = torch.randn(2, 28, 28, 256, generator=g).to(torch.bfloat16).to(gpu)
    before = out.clone()
    conv_op(x, w, pad=(1, 1), x_off=128, cin=128, act=1, y=out, y_off=64, tile=N.FR_TILE_IMG28)
    _close(out[..., 64:192], conv_ref(x, w, pad=(1, 1), x_off=128, cin=128, act=1))
    assert torch.equal(out[..., :64], before[..., :64]) and torch.equal(out[..., 192:], before[..., 192:])
    x14 = torch.randn(2, 14, 14, 128, generator=g).to(torch.bfloat16).to(gpu)
    with pytest.raises(RuntimeError, match="img28"):
        conv_op(x14, w, pad=(1, 1), tile=N.FR_TILE_IMG28)


def test_conv_residual_prelu_dual_output(gpu):
    g = torch.Generator().manual_seed(5)
    B, H, Cin, Cout = 2, 14, 128, 128
    x = torch.randn(B, H, H, Cin, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / np.sqrt(Cin * 9)
    bias = torch.randn(Cout, generator=g) * 0.1
    slope = torch.rand(Cout, generator=g) * 0.5
    res = torch.randn(B, 7, 7, Cout, generator=g).to(torch.bfloat16).to(gpu)
    s = torch.rand(Cout, generator=g) + 0.5
    t = torch.randn(Cout, generator=g) * 0.1
    y2 = torch.zeros(B, 7, 7, Cout, dtype=torch.bfloat16, device=gpu)
    y = conv_op(x, w, stride=(2, 2), pad=(1, 1), bias=bias, act=2, slope=slope, res=res, y2=y2, aff_s=s, aff_b=t)
    ref = conv_ref(x, w, stride=(2, 2), pad=(1, 1), bias=bias, act=2, slope=slope, res=res)
    _close(y, ref)
    _close(y2, y.float().cpu() * s + t)


def test_conv_channel_slices(gpu):
    """Concat-free Inception wiring: read channels [32:64) of a 160-ch buffer, write [96:128)."""
    g = torch.Generator().manual_seed(9)
    B, H = 2, 17
    buf = torch.randn(B, H, H, 160, generator=g).to(torch.bfloat16).to(gpu)
    before = buf.clone()
    w = torch.randn(32, 32, 3, 3, generator=g) / 17
    conv_op(buf.clone(), w, pad=(1, 1), x_off=32, cin=32, act=1, y=buf, y_off=96)
    ref = conv_ref(before, w, pad=(1, 1), x_off=32, cin=32, act=1)
    _close(buf[..., 96:128], ref)
    assert torch.equal(buf[..., :96], before[..., :96]) and torch.equal(buf[..., 128:], before[..., 128:])


@pytest.mark.parametrize("split", [2, 5])
def test_conv_split_k(gpu, split):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 7, 7, 512, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(512, 512, 3, 3, generator=g) / 68
    res = torch.randn(2, 7, 7, 512, generator=g).to(torch.bfloat16).to(gpu)
    y = conv_op(x, w, pad=(1, 1), res=res, act=1, split_k=split)
    _close(y, conv_ref(x, w, pad=(1, 1), res=res, act=1))


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_preprocess_u8_and_f32(gpu, dtype):
    """q = 255 * Normalize(ToTensor(u)) = 2u - 255, exact, duplicated into channels 3..5."""
    rng = np.random.default_rng(0)
    u8 = rng.integers(0, 256, (3, 9, 11, 3), dtype=np.uint8)
    xin = torch.from_numpy(u8).to(gpu)
    dt = N.FR_DTYPE[dtype]
    out = torch.empty(3, 9, 11, 8, dtype=TORCH_DT[dtype], device=gpu)
    N.check(N.lib().fr_op_preprocess(xin.data_ptr(), N.FR_IN_U8_NHWC, 3, 9, 11, out.data_ptr(), dt, N.stream_ptr()))
    torch.cuda.synchronize()
    q = 2 * torch.from_numpy(u8).float() - 255
    assert torch.equal(out[..., :3].float().cpu(), q) and torch.equal(out[..., 3:6].float().cpu(), q)
    assert torch.count_nonzero(out[..., 6:]) == 0
    ref = (torch.from_numpy(u8).float().div(255) - 0.5) / 0.5  # ToTensor + Normalize(0.5, 0.5)
    f = ref.permute(0, 3, 1, 2).contiguous().to(gpu)
    out2 = torch.empty_like(out)
    N.check(N.lib().fr_op_preprocess(f.data_ptr(), N.FR_IN_F32_NCHW, 3, 9, 11, out2.data_ptr(), dt, N.stream_ptr()))
    torch.cuda.synchronize()
    assert torch.allclose(out2.float(), out.float(), atol=0.5)


@pytest.mark.parametrize("k,s,p,H", [(3, 2, 1, 56), (3, 2, 0, 77), (3, 2, 0, 17)])
def test_maxpool(gpu, k, s, p, H):
    x = torch.randn(2, H, H, 64).to(torch.bfloat16).to(gpu)
    Ho = (H + 2 * p - k) // s + 1
    y = torch.zeros(2, Ho, Ho, 128, dtype=torch.bfloat16, device=gpu)
    N.check(N.lib().fr_op_maxpool(x.data_ptr(), 2, H, H, 64, 0, 64, k, s, p, y.data_ptr(), 128, 64, Ho, Ho,
                                  0, N.stream_ptr()))
    torch.cuda.synchronize()
    ref = torch.nn.functional.max_pool2d(x.float().cpu().permute(0, 3, 1, 2), k, s, p).permute(0, 2, 3, 1)
    assert torch.equal(y[..., 64:].float().cpu(), ref)
    assert torch.count_nonzero(y[..., :64]) == 0


def test_avgpool(gpu):
    x = torch.randn(3, 4, 4, 2048).to(torch.bfloat16).to(gpu)
    y = torch.empty(3, 2048, dtype=torch.bfloat16, device=gpu)
    N.check(N.lib().fr_op_avgpool(x.data_ptr(), 3, 4, 4, 2048, y.data_ptr(), 0, N.stream_ptr()))
    torch.cuda.synchronize()
    _close(y, x.float().cpu().mean(dim=(1, 2)), tol=8e-3)


@pytest.mark.parametrize("B,K,split,norm", [(5, 2048, 4, 1), (256, 25088, 32, 1), (7, 1792, 1, 0)])
def test_linear_head(gpu, B, K, split, norm):
    from tests.helpers import pack_weight
    g = torch.Generator().manual_seed(B)
    x = torch.randn(B, K, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(512, K, generator=g) / np.sqrt(K)
    b = torch.randn(512, generator=g) * 0.1
    wp, npad, kpad = pack_weight(w.view(512, K, 1, 1), gpu)
    bd = b.to(gpu)
    out = torch.empty(B, 512, device=gpu)
    part = torch.empty(split * B * npad, device=gpu)
    N.check(N.lib().fr_op_linear(x.data_ptr(), B, K, wp.data_ptr(), 512, npad, kpad, bd.data_ptr(), norm,
                                 out.data_ptr(), split, part.data_ptr(), 0, N.stream_ptr()))
    torch.cuda.synchronize()
    ref = x.float().cpu() @ bf16_round(w).t() + b
    if norm:
        ref = torch.nn.functional.normalize(ref, dim=1)
    assert torch.allclose(out.cpu(), ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())


# ------------------------------------------------------------------------------ match
def _np_topk(P, G, k):
    """oracle: notebook np.dot + stable (score desc, index asc) order."""
    from oracle.match import topk_dot
    return topk_dot(P, G, k)


def _norm(a):
    return (a / np.linalg.norm(a, axis=1, keepdims=True)).astype(np.float32)


@pytest.mark.parametrize("B,Ng,k", [(256, 10000, 5), (3, 1000, 1), (70, 130, 16), (1, 64, 8), (65, 4097, 5)])
def test_match_topk(gpu, B, Ng, k):
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(B + Ng)
    G = _norm(rng.standard_normal((Ng, 512)))
    P = _norm(rng.standard_normal((B, 512)))
    P[: min(B, Ng)] = _norm(G[: min(B, Ng)] + 0.05 * rng.standard_normal((min(B, Ng), 512)))  # planted
    gal = DeviceGallery(G)
    s, i = gal.search(P, k)
    rs, ri = _np_topk(P, G, k)
    assert np.allclose(s, rs, atol=1e-5)
    kk = min(k, Ng)
    gap_ok = np.ones_like(ri, dtype=bool)
    gap_ok[:, :-1] = (rs[:, :-1] - rs[:, 1:]) > 1e-5  # only compare positions separated by a real gap
    assert np.array_equal(i[:, :kk][gap_ok[:, :kk]], ri[:, :kk][gap_ok[:, :kk]])
    assert np.array_equal(i[:, 0], ri[:, 0])


def test_match_ties_lowest_index(gpu):
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(3)
    base = _norm(rng.standard_normal((50, 512)))
    G = np.concatenate([base, base, base], 0)  # every row present 3x: exact score ties
    gal = DeviceGallery(G)
    s, i = gal.search(base[:10], 3)
    for r in range(10):
        assert list(i[r]) == [r, r + 50, r + 100], i[r]
        assert s[r, 0] == s[r, 1] == s[r, 2]


def test_match_ties_across_splits_multi_tile(gpu):
    """The D = 512 register-probe kernel (several 64-row tiles per split, 4 sub-lists per probe) and the
    merge keep the (score desc, index asc) order for exact ties spread over tiles and splits."""
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(21)
    Ng = 20000
    G = _norm(rng.standard_normal((Ng, 512)))
    dup = [5, 4999, 10007, 15013, 19999]  # copies of row 5: other tiles, other splits, the last row
    for r in dup[1:]:
        G[r] = G[5]
    P = _norm(rng.standard_normal((256, 512)))
    P[:40] = _norm(G[5] + 0.02 * rng.standard_normal((40, 512)))
    gal = DeviceGallery(G)
    s, i = gal.search(P, 8)
    rs, ri = _np_topk(P, G, 8)
    for r in range(40):
        assert list(i[r, :5]) == dup, i[r]
        assert len(set(s[r, :5].tolist())) == 1
    assert np.array_equal(i[:, 0], ri[:, 0])
    assert np.allclose(s, rs, atol=1e-5)


@pytest.mark.parametrize("Ng,k", [(10000, 5), (777, 8), (40000, 5), (70000, 1)])
def test_match_small_batch_rows_kernel(gpu, Ng, k):
    """B <= 4 takes match_rows_kernel (one wave per 64 rows, exact_dot's fmaf order): its scores equal the
    MFMA kernels' (B = 9 runs match_p512 below 32768 rows, the bf16x3 path + exact rescoring above) bit for bit,
    ties keep (score desc, index asc) across waves (recognition_engine.py:277-289 order), and the indices match
    the numpy oracle."""
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(Ng + k)
    G = _norm(rng.standard_normal((Ng, 512)))
    for r in (Ng // 3, Ng // 2, Ng - 1):  # exact ties with row 7 in other waves / lists
        G[r] = G[7]
    P = _norm(rng.standard_normal((9, 512)))
    P[0] = _norm(G[7:8] + 0.02 * rng.standard_normal((1, 512)))[0]
    P[2] = _norm(G[100:101] + 0.05 * rng.standard_normal((1, 512)))[0]
    gal = DeviceGallery(G)
    s9, i9 = gal.search(P, k)
    for B in (1, 2, 3, 4):
        s, i = gal.search(P[:B], k)
        assert np.array_equal(s, s9[:B]) and np.array_equal(i, i9[:B]), B
    rs, ri = _np_topk(P, G, k)
    assert np.array_equal(i9[:, 0], ri[:, 0])
    assert np.allclose(s9, rs, atol=1e-5)
    assert list(i9[0, : min(k, 4)]) == [7, Ng // 3, Ng // 2, Ng - 1][: min(k, 4)]


def test_match_unnormalized_rows_cosine(gpu):
    """cosine_similarity semantics: non-unit rows are divided by their norm, zero rows score 0."""
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(4)
    G = rng.standard_normal((20, 512)).astype(np.float32) * 3.0
    G[7] = 0
    P = _norm(rng.standard_normal((2, 512)))
    gal = DeviceGallery(G)
    s, i = gal.search(P, 16)
    ref = P @ _norm(np.where(np.linalg.norm(G, axis=1, keepdims=True) == 0, 1, G)).T
    ref[:, 7] = 0
    for r in range(2):
        assert np.allclose(s[r], np.sort(ref[r])[::-1][:16], atol=1e-5)


def test_topk_merge(gpu):
    rng = np.random.default_rng(8)
    B, L, k = 9, 6, 5
    cs = np.sort(rng.standard_normal((B, L, k)).astype(np.float32), axis=2)[:, :, ::-1].copy()
    ci = rng.permutation(B * L * k).reshape(B, L, k).astype(np.int32)
    cs[0, 1, 0] = cs[0, 0, 0] = 9.0  # tie across lists → lower index first
    tcs, tci = torch.from_numpy(cs).to(gpu), torch.from_numpy(ci).to(gpu)
    os_, oi = torch.empty(B, k, device=gpu), torch.empty(B, k, dtype=torch.int32, device=gpu)
    N.check(N.lib().fr_topk_merge(tcs.data_ptr(), tci.data_ptr(), B, L, k, os_.data_ptr(), oi.data_ptr(),
                                  N.stream_ptr()))
    torch.cuda.synchronize()
    for b in range(B):
        cand = sorted(zip(cs[b].ravel().tolist(), ci[b].ravel().tolist()), key=lambda t: (-t[0], t[1]))[:k]
        assert oi[b].cpu().tolist() == [c[1] for c in cand]
        assert np.allclose(os_[b].cpu().numpy(), [c[0] for c in cand])


@pytest.mark.parametrize("W,B,k", [(8, 2048, 5), (2, 9, 16), (3, 1, 1)])
def test_topk_merge_ranks_equals_list_merge(gpu, W, B, k):
    """fr_topk_merge_ranks over the all-gathered exchange block [W][2][B][k] (scores, then indices: the
    one-collective candidate exchange of ShardedMatcher) equals fr_topk_merge of the same lists in its
    [B][W][k] layout, bit for bit, including exact ties across ranks and -inf / -1 padding."""
    rng = np.random.default_rng(W * 100 + k)
    cs = np.sort(rng.standard_normal((W, B, k)).astype(np.float32), axis=2)[:, :, ::-1].copy()
    ci = rng.permutation(W * B * k).reshape(W, B, k).astype(np.int32)
    if W > 1:
        cs[1, 0, 0] = cs[0, 0, 0] = 9.0  # tie across ranks -> lower index first
    cs[-1, -1, -1], ci[-1, -1, -1] = -np.inf, -1  # a short shard's padding
    x = np.empty((W, 2, B, k), np.int32)
    x[:, 0] = cs.view(np.int32)
    x[:, 1] = ci
    tx = torch.from_numpy(x).to(gpu)
    s1, i1 = torch.empty(B, k, device=gpu), torch.empty(B, k, dtype=torch.int32, device=gpu)
    N.check(N.lib().fr_topk_merge_ranks(tx.data_ptr(), W, B, k, s1.data_ptr(), i1.data_ptr(), N.stream_ptr()))
    tcs = torch.from_numpy(np.ascontiguousarray(cs.transpose(1, 0, 2))).to(gpu)
    tci = torch.from_numpy(np.ascontiguousarray(ci.transpose(1, 0, 2))).to(gpu)
    s2, i2 = torch.empty(B, k, device=gpu), torch.empty(B, k, dtype=torch.int32, device=gpu)
    N.check(N.lib().fr_topk_merge(tcs.data_ptr(), tci.data_ptr(), B, W, k, s2.data_ptr(), i2.data_ptr(), N.stream_ptr()))
    torch.cuda.synchronize()
    assert torch.equal(s1, s2) and torch.equal(i1, i2)
    from oracle.match import merge_topk
    rs, ri = merge_topk(cs.transpose(1, 0, 2), ci.transpose(1, 0, 2), k)
    assert np.array_equal(i1.cpu().numpy(), ri.astype(np.int32)) and np.array_equal(s1.cpu().numpy(), rs)


def test_segment_mean_normalize(gpu):
    rng = np.random.default_rng(2)
    E = _norm(rng.standard_normal((10, 512)))
    seg = np.array([0, 3, 4, 10], np.int32)
    te, ts = torch.from_numpy(E).to(gpu), torch.from_numpy(seg).to(gpu)
    out = torch.empty(3, 512, device=gpu)
    N.check(N.lib().fr_segment_mean_normalize(te.data_ptr(), 512, ts.data_ptr(), 3, out.data_ptr(), N.stream_ptr()))
    torch.cuda.synchronize()
    from oracle.match import folder_mean
    for s in range(3):
        ref = folder_mean(E[seg[s]:seg[s + 1]])
        assert np.allclose(out[s].cpu().numpy(), ref, atol=1e-6)


def _border_class(H, W):
    rc = torch.ones(H, dtype=torch.long)
    rc[0], rc[-1] = 0, 2
    cc = torch.ones(W, dtype=torch.long)
    cc[0], cc[-1] = 0, 2
    return 3 * rc[:, None] + cc[None, :]


BIAS9_CASES = [(2, 14, 14, 256, 256, None), (2, 14, 14, 256, 256, N.FR_TILE_BAND), (2, 28, 28, 128, 128, None),
               (2, 56, 56, 64, 64, 2), (2, 28, 28, 128, 128, 0), (2, 28, 28, 128, 128, N.FR_TILE_IMG28),
               (2, 56, 56, 64, 64, N.FR_TILE_IMG56), (2, 56, 56, 64, 64, N.FR_TILE_ROWS),
               (1, 112, 112, 64, 64, N.FR_TILE_ROWS), (2, 56, 56, 64, 128, N.FR_TILE_ROWS)]


@pytest.mark.parametrize("case", BIAS9_CASES)
def test_conv_bias9_prefolded_bn(gpu, case):
    """Pre-conv BN folded into a 3x3/s1/p1 conv: bias9[border class] replaces bias (every kernel path:
    band, igemm tiles, split-K reduce).  Reference: conv(pad0(s*x + t)) in f32."""
    B, H, W, C, Cout, tile = case
    g = torch.Generator().manual_seed(H + C)
    x = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn(Cout, C, 3, 3, generator=g) / np.sqrt(C * 9)
    s = torch.rand(C, generator=g) + 0.5
    t = torch.randn(C, generator=g)
    slope = torch.rand(Cout, generator=g) * 0.5
    wf = w * s[None, :, None, None]
    T = torch.einsum("ocrs,c->ors", w, t)
    valid = [(1, 2), (0, 1, 2), (0, 1)]
    b9 = torch.stack([T[:, list(valid[rc])][:, :, list(valid[cc])].sum((1, 2)) for rc in range(3) for cc in range(3)])
    y = conv_op(x, wf, pad=(1, 1), act=2, slope=slope, bias9=b9, tile=tile)
    xf = x.float().cpu().permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(xf * s[None, :, None, None] + t[None, :, None, None], q16(w), padding=1)
    ref = torch.nn.functional.prelu(ref, slope).permute(0, 2, 3, 1)
    got = y.float().cpu()
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-2, err
    # border rows/cols really use their own class (a wrong class would be off by O(|T|))
    cls = _border_class(H, W)
    assert set(cls.unique().tolist()) == set(range(9))


@pytest.mark.parametrize("B,Ng,k", [(256, 10000, 5), (2048, 20000, 5), (33, 5000, 16), (1, 4096, 1)])
def test_match_x3_equals_exact(gpu, B, Ng, k):
    """bf16x3 candidates + exact rescoring (match_x3.hip) == the f32-MFMA kernel, bit for bit."""
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(B * 7 + Ng)
    G = _norm(rng.standard_normal((Ng, 512)))
    P = _norm(rng.standard_normal((B, 512)))
    m = min(B, Ng) // 2
    P[:m] = _norm(G[:m] + 0.05 * rng.standard_normal((m, 512)))
    gal = DeviceGallery(G, x3_min_rows=4096)
    s3, i3 = gal.search(P, k)
    gal.set_exact(True)
    se, ie = gal.search(P, k)
    assert np.array_equal(i3, ie)
    assert np.array_equal(s3, se)  # identical f32 fmaf chains
    rs, ri = _np_topk(P, G, k)
    assert np.allclose(s3, rs, atol=1e-5)
    gal.close()


@pytest.mark.parametrize("ndup,rescan", [(40, False), (70, True)])
def test_match_x3_fallback_on_ties(gpu, ndup, rescan):
    """ndup identical copies of a row, one per 64-row tile (at 6000 rows and 6 probes every tile is its own
    gallery split, so no candidate sub-list overflows): more than KC - k = 27 candidates tie within 2 eps, so the
    32-candidate proof fails.  40 copies are settled by the widened 64-candidate pass (no rescan); 70 copies
    exceed it too and the probe is rescanned exactly.  Either way lowest indices first, like the f32 kernel."""
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(5)
    G = _norm(rng.standard_normal((6000, 512)))
    dups = [64 * t + 5 for t in range(2, 2 + ndup)]
    G[dups] = G[7]
    P = _norm(G[[7, 11]] + 0.01 * rng.standard_normal((2, 512)))
    P = np.concatenate([P, _norm(rng.standard_normal((4, 512)))])  # B > 4: the bf16x3 path, not match_rows
    gal = DeviceGallery(G, x3_min_rows=4096)
    fb0 = gal.fallbacks()
    s3, i3 = gal.search(P, 5)
    assert (gal.fallbacks() - fb0 >= 1) == rescan
    assert list(i3[0]) == [7] + dups[:4]
    gal.set_exact(True)
    se, ie = gal.search(P, 5)
    assert np.array_equal(i3, ie) and np.array_equal(s3, se)
    gal.close()


def test_match_x3_sublist_overflow_floor(gpu):
    """Twelve graded near-duplicates of the probe in rows 16*(i//4) + i%4 -- all in ONE candidate
    sub-list (rows 16j + 4*sub + r of a tile; KP = 8 entries), which overflows: its floor enters the proof.  k = 5 is provable from the candidates (no rescan);
    k = 8 needs the sub-list's own last entry, which is also its floor, so the proof fails and the
    probe is rescanned exactly.  Both equal the exact f32 kernel bit for bit.  (k > 8 is routed to the
    exact kernel by fr_match_topk: test_match_large_k_takes_exact_path.)"""
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(9)
    G = _norm(rng.standard_normal((8192, 512)))
    P = _norm(rng.standard_normal((6, 512)))  # B > 4: the bf16x3 path, not match_rows
    rows = [16 * (i // 4) + i % 4 for i in range(12)]
    for i, r in enumerate(rows):
        G[r] = _norm(P[:1] + (0.1 + 0.05 * i) * _norm(rng.standard_normal((1, 512))))[0]
    gal = DeviceGallery(G, x3_min_rows=4096)
    for k, want_fb in ((5, 0), (8, 1)):
        gal.set_exact(False)
        fb0 = gal.fallbacks()
        s3, i3 = gal.search(P, k)
        assert list(i3[0]) == rows[:k]
        assert gal.fallbacks() - fb0 == want_fb
        gal.set_exact(True)
        se, ie = gal.search(P, k)
        assert np.array_equal(i3, ie) and np.array_equal(s3, se)
    gal.close()


def test_match_large_k_takes_exact_path(gpu):
    """k > KC/2 = 8 goes to the exact f32 kernel on an x3-sized gallery: no candidate pass, no rescans
    (at k = 16 the proof could never pass and every probe fell back to a one-wave rescan)."""
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(12)
    G = _norm(rng.standard_normal((8192, 512)))
    P = _norm(rng.standard_normal((64, 512)))
    gal = DeviceGallery(G, x3_min_rows=4096)
    fb0 = gal.fallbacks()
    s, i = gal.search(P, 16)
    assert gal.fallbacks() == fb0
    rs, ri = _np_topk(P, G, 16)
    assert np.array_equal(i[:, 0], ri[:, 0]) and np.allclose(s, rs, atol=1e-5)
    gal.close()


def _host_top1_f64(P, G, chunk=131_072):
    """Chunked float64 argmax (lowest index on ties) + the gap to the runner-up, per probe."""
    P = P.astype(np.float64)
    best = np.full(len(P), -np.inf)
    second = np.full(len(P), -np.inf)
    arg = np.zeros(len(P), np.int64)
    for c in range(0, len(G), chunk):
        S = P @ G[c:c + chunk].astype(np.float64).T
        a = np.argmax(S, axis=1)
        m = S[np.arange(len(S)), a]
        S[np.arange(len(S)), a] = -np.inf
        m2 = S.max(axis=1) if S.shape[1] > 1 else np.full(len(S), -np.inf)
        upd = m > best
        second = np.where(upd, np.maximum(best, m2), np.maximum(second, m))
        arg, best = np.where(upd, a + c, arg), np.where(upd, m, best)
    return arg, best - second


@pytest.mark.timeout(300)
@pytest.mark.parametrize("B,Ng", [(2048, 125_000), (256, 1_000_000)])
def test_match_config4_per_rank_shapes(gpu, B, Ng):
    """BASELINE config 4's per-rank match shapes (2048 gathered probes x a 125k-row shard, and one rank's
    256 probes x the whole 1M rows) through fr_match_topk's bf16x3 path: equal to the exact f32 kernel
    (FR_OPT_MATCH_EXACT) bit for bit, and top-1 equal to a float64 host argmax wherever the runner-up
    gap exceeds the f32 scoring noise (the near-tie count and the proof fallbacks are reported)."""
    from facerecognition_amd.gallery import DeviceGallery
    from facerecognition_amd.synthetic import synthetic_gallery_rows
    G = synthetic_gallery_rows(0, Ng, gpu, seed=5)
    g = torch.Generator(device=gpu)
    g.manual_seed(B)
    P = torch.randn((B, 512), generator=g, device=gpu)
    plant = torch.arange(B // 4, device=gpu) * (Ng // (B // 4)) + 1
    P[: B // 4] = G[plant] + 0.05 / np.sqrt(512) * P[: B // 4]
    P /= P.norm(dim=1, keepdim=True)
    gal = DeviceGallery(device=0)
    gal.set_device_rows(G)
    fb0 = gal.fallbacks()
    s3, i3 = (t.cpu().numpy() for t in gal.search_device(P, 5))
    fb = gal.fallbacks() - fb0
    gal.set_exact(True)
    se, ie = (t.cpu().numpy() for t in gal.search_device(P, 5))
    assert np.array_equal(i3, ie)
    assert np.array_equal(s3.view(np.uint32), se.view(np.uint32))
    assert np.array_equal(i3[: B // 4, 0], plant.cpu().numpy())
    arg, gap = _host_top1_f64(P.cpu().numpy(), G.cpu().numpy())
    clear = gap > 1e-5
    assert clear.mean() > 0.9
    assert np.array_equal(i3[clear, 0], arg[clear])
    print(f"{B}x{Ng}: bf16x3 == exact f32 bit for bit; {fb} proof fallbacks; "
          f"{int((~clear).sum())} near-tie probes (gap <= 1e-5) of {B}")
    gal.close()


def test_nccl_world1_all_gather(gpu):
    """The RCCL ("nccl") branch of distributed._all_gather (config 4's collective) on a world-1 group on
    the device (RCCL refuses two ranks on one GPU, and the test box has one): all_gather_into_tensor of
    embeddings, then ShardedMatcher's four exchange steps (all-gather, shard top-k, candidate all-gather,
    fr_topk_merge) through RCCL, equal to the plain search bit for bit."""
    import socket
    import torch.distributed as dist
    from facerecognition_amd.distributed import ShardedMatcher, _all_gather
    from facerecognition_amd.gallery import DeviceGallery
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=gpu)
    try:
        assert dist.get_backend() == "nccl"
        x = torch.randn(256, 512, device=gpu)
        out = torch.empty(256, 512, device=gpu)
        _all_gather(out, x)
        torch.cuda.synchronize()
        assert torch.equal(out, x)
        rng = np.random.default_rng(3)
        G = _norm(rng.standard_normal((40_000, 512)))
        gal = DeviceGallery(G)
        P = torch.from_numpy(_norm(rng.standard_normal((64, 512)))).to(gpu)
        m = ShardedMatcher(64, 512, 5, lambda p, s, i: gal.search_device(p, 5, s, i), gpu, always_exchange=True)
        s, i = m.search(P)
        s0, i0 = gal.search_device(P, 5)
        torch.cuda.synchronize()
        assert torch.equal(i, i0) and torch.equal(s, s0)
        rs, ri = _np_topk(P.cpu().numpy(), G, 5)
        assert np.array_equal(i.cpu().numpy()[:, 0], ri[:, 0])
        gal.close()
    finally:
        dist.destroy_process_group()


# ------------------------------------------------------------------------------ match, k > 16
@pytest.mark.parametrize("B,Ng,k", [(5, 20000, 17), (3, 20000, 100), (2, 5000, 1000), (1, 9000, 4096), (4, 300, 700)])
def test_match_large_k(gpu, B, Ng, k):
    """k > 16 (IndexFlatIP.search with any k): exact score rows + device radix select, against the
    oracle's (score desc, index asc) order; rows past the gallery end are (-inf, -1)."""
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(B * 7 + Ng + k)
    G = _norm(rng.standard_normal((Ng, 512)))
    G[Ng // 2] = G[1]  # an exact tie
    P = _norm(rng.standard_normal((B, 512)))
    P[0] = _norm((G[1] + 0.01 * rng.standard_normal(512))[None])[0]
    gal = DeviceGallery(G)
    s, i = gal.search(P, k)
    rs, ri = _np_topk(P, G, k)
    kk = min(k, Ng)
    assert np.all(np.diff(s[:, :kk], axis=1) <= 0)
    assert np.allclose(s[:, :kk], rs[:, :kk], atol=1e-5)
    gap_ok = np.ones((B, kk), dtype=bool)
    gap_ok[:, :-1] = (rs[:, :kk - 1] - rs[:, 1:kk]) > 1e-5
    gap_ok[:, 1:] &= gap_ok[:, :-1].copy() | ((rs[:, :kk - 1] - rs[:, 1:kk]) > 1e-5)
    assert np.array_equal(i[:, :kk][gap_ok], ri[:, :kk][gap_ok])
    assert list(i[0, :2]) == [1, Ng // 2] and s[0, 0] == s[0, 1]  # the tie: lower index first
    if k > Ng:
        assert np.all(s[:, Ng:] == -np.inf) and np.all(i[:, Ng:] == -1)
    # the small-k list is a prefix of the large-k list, bit for bit (the same MFMA score sequence)
    s16, i16 = gal.search(P, 16)
    m = min(16, kk)
    assert np.array_equal(s[:, :m], s16[:, :m]) and np.array_equal(i[:, :m], i16[:, :m])
    gal.close()


def test_match_large_k_x3_gallery_prefix(gpu):
    """On a gallery that takes the bf16x3 path for small k (>= X3_MIN_ROWS rows), the large-k list still
    starts with the small-k list (the x3 path rescores exactly)."""
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(5)
    G = _norm(rng.standard_normal((40000, 512)))
    P = _norm(rng.standard_normal((8, 512)))
    P[:4] = _norm(G[:4] + 0.05 * rng.standard_normal((4, 512)))
    gal = DeviceGallery(G)
    s5, i5 = gal.search(P, 5)
    s, i = gal.search(P, 64)
    gal.close()
    assert np.array_equal(i[:, :5], i5) and np.array_equal(s[:, :5], s5)


def test_recognize_with_faiss_large_k(gpu, tmp_path):
    """recognize_with_faiss with k = 40 > 16 against oracle.match.faiss_flat_ip_search."""
    from facerecognition_amd import extract_embeddings as EE
    from facerecognition_amd.recognition_engine import RecognitionEngine
    from oracle.match import faiss_flat_ip_search
    rng = np.random.default_rng(8)
    protos = _norm(rng.standard_normal((300, 512)))
    EE.build_faiss_index(protos, str(tmp_path / "idx.faiss"))
    eng = RecognitionEngine.__new__(RecognitionEngine)  # only the FAISS state: no model, no db
    eng.threshold, eng.id_to_label, eng.faiss_index, eng.prototypes = 0.5, None, None, None
    eng._load_faiss(str(tmp_path / "idx.faiss"))
    assert eng.faiss_index is not None
    probe = protos[17] + 0.02 * rng.standard_normal(512).astype(np.float32)
    name, score, res = eng.recognize_with_faiss(probe, k=40)
    s_ref, i_ref = faiss_flat_ip_search(protos, probe, 40)
    assert [r[0] for r in res] == [f"ID_{j}" for j in i_ref[0]]
    assert np.allclose([r[1] for r in res], s_ref[0], atol=1e-5)
    assert name == "ID_17"


def test_gallery_write_appends_and_updates_equal_rebuild(gpu):
    """fr_gallery_write: single-row appends (crossing the bf16x3 threshold and several capacity
    doublings), batch appends and in-place row updates give the same top-k, bit for bit, as one
    fr_gallery_set of the final matrix."""
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(17)
    G = _norm(rng.standard_normal((3000, 512)))
    G[100] *= 3.0  # a non-unit row: the norm rule must apply to written rows too
    gal = DeviceGallery(dim=512, x3_min_rows=2048)
    for r in range(1500):
        gal.add(G[r:r + 1])
    gal.add(torch.from_numpy(G[1500:2600]).cuda())  # device rows: crosses x3_min_rows
    gal.add(G[2600:])
    upd = _norm(rng.standard_normal((3, 512)))
    for j, r in enumerate((7, 2047, 2999)):
        G[r] = upd[j]
        gal.update(r, upd[j:j + 1])
    assert gal.ntotal == 3000
    ref = DeviceGallery(G, x3_min_rows=2048)
    P = _norm(rng.standard_normal((64, 512)))
    P[:3] = upd
    for k in (1, 5, 16, 40):
        s, i = gal.search(P, k)
        rs, ri = ref.search(P, k)
        assert np.array_equal(s, rs) and np.array_equal(i, ri), k
    assert list(gal.search(P[:3], 1)[1][:, 0]) == [7, 2047, 2999]
    gal.close()
    ref.close()


def test_gallery_write_after_x3_threshold_raised(gpu):
    """A gallery already split for the bf16x3 path stays on it after FR_OPT_X3_MIN_ROWS is raised, so
    later appends and updates must be split too (else the candidate pass reads stale hi/lo rows and can
    miss new rows): the top-k equals a fresh exact-path gallery of the same rows, bit for bit."""
    from facerecognition_amd import _native as N
    from facerecognition_amd.gallery import DeviceGallery
    rng = np.random.default_rng(23)
    G = _norm(rng.standard_normal((2600, 512)))
    gal = DeviceGallery(G[:2400], x3_min_rows=2048)  # split now
    N.check(N.lib().fr_set_option(gal._h, N.FR_OPT_X3_MIN_ROWS, 1 << 30), "fr_set_option")
    gal.add(G[2400:])  # appends past the (raised) threshold ...
    G[5] = _norm(rng.standard_normal((1, 512)))[0]
    gal.update(5, G[5:6])  # ... and an in-place update
    P = _norm(rng.standard_normal((32, 512)))
    P[:4] = _norm(G[[5, 2400, 2555, 2599]] + 0.01 * rng.standard_normal((4, 512)))
    ref = DeviceGallery(G)
    ref.set_exact(True)
    for k in (1, 5):
        s, i = gal.search(P, k)
        rs, ri = ref.search(P, k)
        assert np.array_equal(s, rs) and np.array_equal(i, ri), k
    assert list(gal.search(P[:4], 1)[1][:, 0]) == [5, 2400, 2555, 2599]
    gal.close()
    ref.close()


SMALL_CASES = [
    # B, H, W, Cin, Cout, stride   (small-batch shapes: bs = 1 layer3 / layer4 / layer2, a transition, bs = 3)
    (1, 14, 14, 256, 256, 1), (1, 7, 7, 512, 512, 1), (1, 28, 28, 128, 256, 2), (1, 28, 28, 128, 128, 1),
    (3, 14, 14, 256, 512, 2), (1, 56, 56, 64, 64, 1)]


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("case", SMALL_CASES)
def test_conv_small(gpu, case, dtype):
    """Small-M implicit GEMM (conv_small.hip, forced): one wave per 16 px x 64 ch over the whole K with the
    igemm's 32-deep MFMA order and epilogue arithmetic, so bias + residual, border-class bias + PReLU and ReLU
    all equal tile 0 bit for bit; a shape it cannot take is refused, never silently run elsewhere."""
    B, H, W, Cin, Cout, st = case
    g = torch.Generator().manual_seed(B + H + Cin + Cout + st + 7)
    x = torch.randn(B, H, W, Cin, generator=g).to(TORCH_DT[dtype]).to(gpu)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / np.sqrt(Cin * 9)
    bias = torch.randn(Cout, generator=g) * 0.1
    slope = torch.rand(Cout, generator=g) * 0.5
    Ho = (H + 2 - 3) // st + 1
    res = torch.randn(B, Ho, Ho, Cout, generator=g).to(TORCH_DT[dtype]).to(gpu)
    kw = dict(stride=(st, st), pad=(1, 1), dtype=dtype)
    y = conv_op(x, w, bias=bias, res=res, tile=N.FR_TILE_SMALL, **kw)
    _close(y, conv_ref(x, w, bias=bias, res=res, **kw), tol=1e-2 if dtype == "bf16" else 2e-3)
    assert torch.equal(y, conv_op(x, w, bias=bias, res=res, tile=0, **kw))
    b9 = torch.randn(9, Cout, generator=g) * 0.1
    y = conv_op(x, w, act=2, slope=slope, bias9=b9, tile=N.FR_TILE_SMALL, **kw)
    assert torch.equal(y, conv_op(x, w, act=2, slope=slope, bias9=b9, tile=0, **kw))
    y = conv_op(x, w, bias=bias, act=1, tile=N.FR_TILE_SMALL, **kw)
    assert torch.equal(y, conv_op(x, w, bias=bias, act=1, tile=0, **kw))
    for ks in (4, 8):  # K split over 4 / 8 waves of a workgroup, summed through LDS in wave order
        y = conv_op(x, w, bias=bias, res=res, tile=N.FR_TILE_SMALL, split_k=ks, **kw)
        _close(y, conv_ref(x, w, bias=bias, res=res, **kw), tol=1e-2 if dtype == "bf16" else 2e-3)
        assert torch.equal(y, conv_op(x, w, bias=bias, res=res, tile=N.FR_TILE_SMALL, split_k=ks, **kw))
        y = conv_op(x, w, act=2, slope=slope, bias9=b9, tile=N.FR_TILE_SMALL, split_k=ks, **kw)
        _close(y, conv_op(x, w, act=2, slope=slope, bias9=b9, tile=0, **kw), tol=1e-2 if dtype == "bf16" else 2e-3)
        # the narrower tiles (32 / 16 output channels, split_k = KS | NF << 8) chunk K by KS alone: the same bits
        for nf in (2, 1):
            yn = conv_op(x, w, bias=bias, res=res, tile=N.FR_TILE_SMALL, split_k=ks | nf << 8, **kw)
            assert torch.equal(yn, conv_op(x, w, bias=bias, res=res, tile=N.FR_TILE_SMALL, split_k=ks, **kw))
            yn = conv_op(x, w, act=2, slope=slope, bias9=b9, tile=N.FR_TILE_SMALL, split_k=ks | nf << 8, **kw)
            assert torch.equal(yn, y)
    y16 = conv_op(x, w, bias=bias, act=1, tile=N.FR_TILE_SMALL, split_k=16 | 1 << 8, **kw)
    _close(y16, conv_op(x, w, bias=bias, act=1, tile=0, **kw), tol=1e-2 if dtype == "bf16" else 2e-3)
    with pytest.raises(RuntimeError, match="small"):  # Cout % 64 != 0 for the 64-channel tile
        conv_op(x, torch.randn(32, Cin, 3, 3, generator=g), pad=(1, 1), tile=N.FR_TILE_SMALL, dtype=dtype)
    with pytest.raises(RuntimeError, match="small"):  # no 16-wave split of the 64-channel tile
        conv_op(x, w, pad=(1, 1), tile=N.FR_TILE_SMALL, split_k=16, dtype=dtype)
    w32 = torch.randn(32, Cin, 3, 3, generator=g) / np.sqrt(Cin * 9)  # 32 channels: the 32 / 16-channel tiles
    y32 = conv_op(x, w32, bias=bias[:32], act=1, tile=N.FR_TILE_SMALL, split_k=8 | 2 << 8, **kw)
    assert torch.equal(y32, conv_op(x, w32, bias=bias[:32], act=1, tile=N.FR_TILE_SMALL, split_k=8 | 1 << 8, **kw))
    for sp in (1 | 2 << 8, 1 | 1 << 8):  # one wave per 16 px x 32 / 16 ch over the whole K: tile 0's bits
        assert torch.equal(conv_op(x, w32, bias=bias[:32], act=1, tile=N.FR_TILE_SMALL, split_k=sp, **kw),
                           conv_op(x, w32, bias=bias[:32], act=1, tile=0, **kw))
        assert torch.equal(conv_op(x, w, act=2, slope=slope, bias9=b9, tile=N.FR_TILE_SMALL, split_k=sp, **kw),
                           conv_op(x, w, act=2, slope=slope, bias9=b9, tile=0, **kw))
    _close(y32, conv_ref(x, w32, bias=bias[:32], act=1, **kw), tol=1e-2 if dtype == "bf16" else 2e-3)
