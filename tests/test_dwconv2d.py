"""kernels/dwconv2d counterpart (accunet/dwconv2d.py, csrc/dwconvk.hip).

Pinning: the reference's own known-answer check (kernels/dwconv2d/check.py:18-54:
three dilated 3x3 replicate-padded depthwise convs summed == one 11x11 kernel
through the custom conv) is run on the oracle restatement (CPU) and on the HIP
kernel (GPU). The oracle's replicate path is also checked against torch's
padding_mode="replicate" conv. The GPU kernels are compared with the oracle in
fp64 for the forward and with torch autograd through the oracle for dx, dw, db
(the reference's own backward is not runnable: its bindings are commented out)."""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import accunet_oracle as O  # noqa: E402

from accunet.dwconv2d import replicate_mode  # noqa: E402


def _check_py_weights(g, dim, dtype=torch.float32):
    """The 3 dilated 3x3 convs of check.py and their 11x11 composition (:35-57)."""
    k1 = torch.randn(dim, 1, 3, 3, generator=g).to(dtype)
    k2 = torch.randn(dim, 1, 3, 3, generator=g).to(dtype)
    k3 = torch.randn(dim, 1, 3, 3, generator=g).to(dtype)
    w = torch.zeros(dim, 1, 11, 11, dtype=dtype)
    w[:, :, 4:7, 4:7] = k1
    for a in range(3):
        for b in range(3):
            w[:, :, 2 + 3 * a, 2 + 3 * b] += k2[:, :, a, b]
            w[:, :, 5 * a, 5 * b] += k3[:, :, a, b]
    return k1, k2, k3, w


def test_check_py_kat_on_oracle():
    g = torch.Generator().manual_seed(0)
    x = torch.rand(2, 16, 32, 32, generator=g, dtype=torch.float64)
    k1, k2, k3, w = _check_py_weights(g, 16, torch.float64)
    ref = 0
    for k, d in ((k1, 1), (k2, 3), (k3, 5)):
        conv = torch.nn.Conv2d(16, 16, 3, dilation=d, padding=d, groups=16, padding_mode="replicate",
                               bias=False).double()
        conv.weight.data.copy_(k)
        ref = ref + conv(x)
    out = O.dwconvk(x, w, None, 5, 5, replicate=True)
    assert (out - ref).abs().max().item() < 1e-12


def test_oracle_replicate_matches_torch_replicate_conv():
    g = torch.Generator().manual_seed(1)
    for k, p in ((5, 2), (7, 3), (13, 6)):
        x = torch.randn(2, 4, 20, 24, generator=g, dtype=torch.float64)
        w = torch.randn(4, 1, k, k, generator=g, dtype=torch.float64)
        conv = torch.nn.Conv2d(4, 4, k, padding=p, groups=4, padding_mode="replicate",
                               bias=False).double()
        conv.weight.data.copy_(w)
        assert (O.dwconvk(x, w, None, p, p, True) - conv(x)).abs().max().item() < 1e-12


def test_dispatch_rule():
    assert not replicate_mode(3, 3, 1, 1, False) and replicate_mode(3, 3, 2, 2, False)
    assert not replicate_mode(3, 3, 2, 2, True) and replicate_mode(5, 5, 2, 2, True)


CASES = [  # (N, C, H, W, kh, kw, ph, pw, bias)
    (2, 8, 16, 16, 3, 3, 1, 1, False),    # zero padding (cudnn route)
    (2, 8, 16, 16, 3, 3, 1, 1, True),     # zero padding (at::conv2d route)
    (2, 8, 16, 16, 3, 3, 2, 2, False),    # replicate (custom kernel, 3x3 pad 2)
    (2, 6, 20, 18, 5, 5, 2, 2, True),
    (1, 4, 32, 32, 11, 11, 5, 5, False),  # check.py's 11x11
    (2, 16, 64, 64, 13, 13, 6, 6, True),  # dwconv_layer.py's example shape (fewer channels)
    (1, 3, 12, 40, 7, 9, 2, 4, True),     # pw > ph: the pad_h window quirk
    (1, 2, 256, 256, 31, 31, 15, 15, True),  # largest kernel, row-tiled staging
    (2, 4, 10, 12, 3, 3, 3, 2, True),     # zero padding wider than k-1: fold path
    (1, 2, 1, 9, 5, 3, 2, 1, False),      # a one-row image: both borders fold onto row 0
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_dwconvk_fwd_bwd_matches_oracle(case):
    from accunet.dwconv2d import DepthwiseFunction
    N, C, H, W, kh, kw, ph, pw, has_b = case
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, 1, kh, kw, generator=g) * 0.2
    b = torch.randn(C, generator=g) if has_b else None
    rep = replicate_mode(kh, kw, ph, pw, has_b)
    xd, wd = x.double().requires_grad_(True), w.double().requires_grad_(True)
    bd = b.double().requires_grad_(True) if has_b else None
    ref = O.dwconvk(xd, wd, bd, ph, pw, rep)
    gy = torch.randn(ref.shape, generator=g)
    ref.backward(gy.double())
    dev = "cuda"
    xg, wg = x.to(dev).requires_grad_(True), w.to(dev).requires_grad_(True)
    bg = b.to(dev).requires_grad_(True) if has_b else None
    out = DepthwiseFunction.apply(xg, wg, bg, ph, pw, has_b)
    out.backward(gy.to(dev))
    scale = lambda t: max(1.0, t.abs().max().item())
    k = kh * kw
    assert (out.detach().cpu().double() - ref.detach()).abs().max().item() < 1e-5 * scale(ref) * k ** 0.5
    assert (xg.grad.cpu().double() - xd.grad).abs().max().item() < 1e-5 * scale(xd.grad) * k ** 0.5
    tol_w = 1e-5 * scale(wd.grad) * (N * H * W) ** 0.5
    assert (wg.grad.cpu().double() - wd.grad).abs().max().item() < tol_w
    if has_b:
        assert (bg.grad.cpu().double() - bd.grad).abs().max().item() < 1e-5 * scale(bd.grad) * (N * H * W) ** 0.5


@pytest.mark.gpu
def test_check_py_kat_on_hip():
    from accunet.dwconv2d import DepthwiseFunction
    g = torch.Generator().manual_seed(0)
    x = torch.rand(2, 16, 32, 32, generator=g)
    k1, k2, k3, w = _check_py_weights(g, 16)
    ref = 0
    for k, d in ((k1, 1), (k2, 3), (k3, 5)):
        conv = torch.nn.Conv2d(16, 16, 3, dilation=d, padding=d, groups=16, padding_mode="replicate",
                               bias=False)
        conv.weight.data.copy_(k)
        ref = ref + conv(x).detach()
    out = DepthwiseFunction.apply(x.cuda(), w.cuda(), None, 5, 5, False)
    assert (out.cpu() - ref).abs().mean().item() < 1e-6   # check.py prints mean |diff|
    assert (out.cpu() - ref).abs().max().item() < 1e-4
