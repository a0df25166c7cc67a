"""Large-kernel depthwise convolution with the interface of the reference's native
extension kernels/dwconv2d (Dwconv/dwconv_layer.py: DepthwiseFunction, DwConv2d),
running on csrc/dwconvk.hip.

Semantics of the reference (NCHW fp32, stride 1, groups = channels, output
H - kh + 1 + 2 ph by W - kw + 1 + 2 pw):
  * padding mode as its launchers pick it (depthwise_fwd/launch.cu:12-80): zero
    padding for 3x3 kernels (without bias only when padding is 1; with bias always),
    the custom kernel's replicate padding otherwise (kernel.cuh:104-115);
  * DepthwiseFunction.apply(x, w, b, padding_h, padding_w, is_bias) and
    DwConv2d(num_channel, kernel_size, padding, bias=True) with weight
    randn(C, 1, kh, kw) and zero bias (dwconv_layer.py:34-50).
Backward (which the reference declares but cannot run, its dgrad / wgrad / bgrad
bindings being commented out in dwconv2d.cpp:30-52) returns dx, dw and db of that
forward.
"""
from __future__ import annotations

import torch
from torch import nn

from . import kern


def replicate_mode(kh: int, kw: int, ph: int, pw: int, has_bias: bool) -> bool:
    """launch.cu:28 (no bias: 3x3 with padding 1 -> cudnn, zero padding) and :61
    (bias: every 3x3 -> at::conv2d, zero padding); anything else -> the replicate
    kernel."""
    if kh == 3 and kw == 3 and (has_bias or (ph == 1 and pw == 1)):
        return False
    return True


class DepthwiseFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, padding_h, padding_w, is_bias):
        if x.dim() != 4 or w.dim() != 4 or w.shape[1] != 1 or w.shape[0] != x.shape[1]:
            raise RuntimeError("dwconv2d: x (N,C,H,W) and weight (C,1,kh,kw) expected")
        x = x.contiguous()
        w = w.contiguous()
        N, C, H, W = x.shape
        kh, kw = int(w.shape[2]), int(w.shape[3])
        ph, pw = int(padding_h), int(padding_w)
        bias = b.contiguous() if is_bias else None
        rep = replicate_mode(kh, kw, ph, pw, bool(is_bias))
        oh, ow = kern.dwconvk_out_hw(H, W, kh, kw, ph, pw)
        out = torch.empty(N, C, oh, ow, dtype=x.dtype, device=x.device)
        kern.dwconvk_fwd(x, w, bias, out, N, C, H, W, kh, kw, ph, pw, rep)
        ctx.save_for_backward(x, w)
        ctx.cfg = (N, C, H, W, kh, kw, ph, pw, rep, bool(is_bias))
        return out

    @staticmethod
    def backward(ctx, grad):
        x, w = ctx.saved_tensors
        N, C, H, W, kh, kw, ph, pw, rep, is_bias = ctx.cfg
        grad = grad.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        if dx is not None:
            kern.dwconvk_dgrad(grad, w, dx, N, C, H, W, kh, kw, ph, pw, rep)
        dw = torch.empty_like(w)
        db = torch.empty(C, dtype=x.dtype, device=x.device) if is_bias else None
        kern.dwconvk_wgrad(x, grad, dw, db, N, C, H, W, kh, kw, ph, pw, rep)
        return dx, dw, db, None, None, None


class DwConv2d(nn.Module):
    """Dwconv/dwconv_layer.py:34-50."""

    def __init__(self, num_channel, kernel_size, padding, bias=True) -> None:
        super().__init__()
        kernel_size_h, kernel_size_w = kernel_size
        self.padding_h, self.padding_w = padding
        self.weight = nn.Parameter(torch.randn(num_channel, 1, kernel_size_h, kernel_size_w))
        self.is_bias = bias
        if bias:
            self.bias = nn.Parameter(torch.zeros(num_channel))
        else:
            self.bias = None

    def forward(self, x):
        return DepthwiseFunction.apply(x, self.weight, self.bias, self.padding_h, self.padding_w,
                                       self.is_bias)
