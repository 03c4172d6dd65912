"""Op-level helpers for the kernel parity tests: call libfrhip's fr_op_* entry points on torch
tensors, and build the torch fp32 references they are compared against."""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F

from facerecognition_amd import _native as N


def bf16_round(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).float()


TORCH_DT = {"bf16": torch.bfloat16, "f16": torch.float16}


def q16(t: torch.Tensor, dtype: str = "bf16") -> torch.Tensor:
    return t.to(TORCH_DT[dtype]).float()


def pack_weight(w: torch.Tensor, device, dtype: str = "bf16") -> tuple:
    """[Cout, Cin, kh, kw] f32 → 16-bit [Npad, Kpad] (row n, K = (r, s, c) c fastest)."""
    cout, cin, kh, kw = w.shape
    K = kh * kw * cin
    npad = (cout + 127) // 128 * 128
    kpad = (K + 63) // 64 * 64
    m = torch.zeros((npad, kpad), dtype=TORCH_DT[dtype])
    m[:cout, :K] = w.permute(0, 2, 3, 1).reshape(cout, K).to(TORCH_DT[dtype])
    return m.to(device), npad, kpad


def conv_op(x_nhwc, w, *, stride=(1, 1), pad=(0, 0), bias=None, act=0, slope=None, res=None, res_off=0,
            x_off=0, cin=None, y=None, y_off=0, y2=None, aff_s=None, aff_b=None, split_k=1, dtype="bf16",
            tile=None, bias9=None, timed_iters=0):
    """Run fr_op_conv2d. x_nhwc: cuda 16-bit [B,H,W,Cx] of `dtype`; w: cpu f32 [Cout,Cin,kh,kw].
    timed_iters > 0 (tools/conv_bench.py): also relaunch it that many times, timed one by one with
    events on the launching stream; returns (y, [ms, ...])."""
    dev = x_nhwc.device
    assert x_nhwc.dtype == TORCH_DT[dtype]
    B, H, W, Cx = x_nhwc.shape
    cout, cin_w, kh, kw = w.shape
    cin = cin or cin_w
    wp, npad, kpad = pack_weight(w, dev, dtype)
    Ho = (H + 2 * pad[0] - kh) // stride[0] + 1
    Wo = (W + 2 * pad[1] - kw) // stride[1] + 1
    if y is None:
        y = torch.zeros((B, Ho, Wo, cout), dtype=TORCH_DT[dtype], device=dev)
    d = N.FrConvDesc()
    d.x, d.B, d.H, d.W, d.Cx, d.x_off, d.Cin = x_nhwc.data_ptr(), B, H, W, Cx, x_off, cin
    d.w, d.Cout, d.Kh, d.Kw = wp.data_ptr(), cout, kh, kw
    d.stride_h, d.stride_w, d.pad_h, d.pad_w, d.Npad, d.Kpad = stride[0], stride[1], pad[0], pad[1], npad, kpad
    keep = [wp]

    def dptr(t):
        if t is None:
            return None
        t = t.to(dev).float().contiguous()
        keep.append(t)
        return t.data_ptr()

    d.bias = dptr(bias)
    if bias9 is not None:  # [9, Cout] -> [9, Npad]
        b9 = torch.zeros((9, npad), dtype=torch.float32)
        b9[:, :cout] = bias9
        d.bias9 = dptr(b9)
    d.act = act
    d.slope = dptr(slope)
    if res is not None:
        d.res, d.Cres, d.res_off = res.data_ptr(), res.shape[-1], res_off
    d.y, d.Cy, d.y_off = y.data_ptr(), y.shape[-1], y_off
    if y2 is not None:
        d.y2, d.Cy2, d.y2_off = y2.data_ptr(), y2.shape[-1], 0
        d.aff_s, d.aff_b = dptr(aff_s), dptr(aff_b)
    d.Ho, d.Wo = Ho, Wo
    d.dtype = 1 if dtype == "f16" else 0
    d.tile = 0 if tile is None else tile + 1
    part = None
    if split_k > 1:
        part = torch.empty(split_k * B * Ho * Wo * npad, dtype=torch.float32, device=dev)
        d.split_k, d.partial = split_k, part.data_ptr()
    N.check(N.lib().fr_op_conv2d(ctypes.byref(d), N.stream_ptr(dev)), "fr_op_conv2d")
    torch.cuda.synchronize(dev)
    if timed_iters:
        ms = []
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(timed_iters):
            e0.record()
            N.check(N.lib().fr_op_conv2d(ctypes.byref(d), N.stream_ptr(dev)), "fr_op_conv2d")
            e1.record()
            torch.cuda.synchronize(dev)
            ms.append(e0.elapsed_time(e1))
        return y, ms
    return y


def conv_ref(x_nhwc, w, *, stride=(1, 1), pad=(0, 0), bias=None, act=0, slope=None, res=None, x_off=0, cin=None,
             dtype="bf16"):
    """torch fp32 reference on 16-bit-exact operands; returns NHWC f32 (CPU)."""
    cin = cin or w.shape[1]
    x = x_nhwc.float().cpu()[..., x_off:x_off + cin].permute(0, 3, 1, 2)
    wq = q16(w, dtype)
    y = F.conv2d(x, wq, stride=stride, padding=pad)
    if bias is not None:
        y = y + bias.view(1, -1, 1, 1)
    y = y.permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.float().cpu()
    if act == 1:
        y = torch.relu(y)
    elif act == 2:
        y = torch.where(y > 0, y, y * slope.view(1, 1, 1, -1))
    return y
