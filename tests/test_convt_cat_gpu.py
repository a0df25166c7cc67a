"""The decoder's up + concat (ACC_UNet/ACC_UNet.py:637-648: torch.cat([up(x), skip],
dim=1) with up = ConvTranspose2d(k=2, s=2)) as one shuffle-and-concat pass
(ops.conv_transpose2x2_cat, accunet_convt_cat) against the two-step form it replaces
(ops.conv_transpose2x2, then ops.cat_channels) and against torch's NCHW ops in fp64."""
import os
import sys

import pytest
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "acc-unet-unext_amd"))

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("B,H,W,Ci,Co,Cs", [(2, 8, 8, 64, 32, 32), (3, 5, 7, 16, 8, 12),
                                            (16, 32, 32, 64, 32, 32), (1, 4, 6, 512, 256, 256)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_convt_cat_matches_two_step_and_torch(B, H, W, Ci, Co, Cs, dt):
    from accunet import ops
    g = torch.Generator().manual_seed(B * 100 + H + Co)
    x = torch.randn(B, H, W, Ci, generator=g)
    skip = torch.randn(B, 2 * H, 2 * W, Cs, generator=g)
    w = torch.randn(Ci, Co, 2, 2, generator=g) * Ci ** -0.5
    b = torch.randn(Co, generator=g) * 0.1
    gy = torch.randn(B, 2 * H, 2 * W, Co + Cs, generator=g)
    outs = {}
    for name, fn in (("fused", lambda xx, ww, bb, ss: ops.conv_transpose2x2_cat(xx, ww, bb, ss)),
                     ("two_step", lambda xx, ww, bb, ss: ops.cat_channels(
                         ops.conv_transpose2x2(xx, ww, bb), ss))):
        xx = x.to(DEV, dt).requires_grad_(True)
        ss = skip.to(DEV, dt).requires_grad_(True)
        ww = w.to(DEV).requires_grad_(True)
        bb = b.to(DEV).requires_grad_(True)
        y = fn(xx, ww, bb, ss)
        (y.float() * gy.to(DEV)).sum().backward()
        torch.cuda.synchronize()
        outs[name] = [t.detach().float().cpu() for t in (y, xx.grad, ss.grad, ww.grad, bb.grad)]
    f, t2 = outs["fused"], outs["two_step"]
    # the same shuffled values, bias adds, GEMMs and copies: bit for bit (the bias gradient
    # sums dT instead of dY: the same terms in another order)
    for i in range(4):
        assert torch.equal(f[i], t2[i]), i
    assert torch.allclose(f[4], t2[4], rtol=1e-5, atol=1e-5 * float(t2[4].abs().max()))
    # torch fp64 reference (NCHW)
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    sr = skip.double().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    yr = torch.cat([F.conv_transpose2d(xr, wr, br, stride=2), sr], dim=1)
    (yr * gy.double().permute(0, 3, 1, 2)).sum().backward()
    ref = [yr.detach().permute(0, 2, 3, 1), xr.grad.permute(0, 2, 3, 1), sr.grad.permute(0, 2, 3, 1),
           wr.grad, br.grad]
    tol = 2e-5 if dt == torch.float32 else 3e-2
    for i, (a, r) in enumerate(zip(f, ref)):
        err = float((a.double() - r).abs().max())
        assert err <= tol * (float(r.abs().max()) + 1.0), (i, err)
