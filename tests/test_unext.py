"""UNeXt (Experiments/nets/UNext.py) on the HIP kernels (accunet/unext.py) against the
oracle restatement (oracle/accunet_oracle.py: unext_forward).

The reference module imports timm / torchvision, which this image lacks; the fixture
tests/golden/unext.npz was recorded by running the reference module itself with import
shims for them (tests/golden/make_golden.py: ref_unext; to_2tuple restated, init-only
trunc_normal_, DropPath never built at drop_path_rate 0), and pins the oracle
(test_oracle_golden.py: test_unext_matches_reference) and, below, the HIP model's eval
output at 64^2 and at the Cfg5 resolution 224^2. The oracle's pieces are also
cross-checked against torch here (shift vs an independent index formula, bilinear x2
vs F.interpolate). The HIP path is held to
the fp64 oracle within 4x the reference's own fp32 error (the oracle run in fp32 on
one-rounding-perturbed inputs) plus 1e-4 of each tensor's scale, like the ACC-UNet
whole-model tests."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import parity_util as PU  # noqa: E402
from parity_util import O  # noqa: E402

BUF = ("running_mean", "running_var", "num_batches_tracked")


def test_state_dict_matches_oracle_spec():
    from accunet.unext import UNext
    m = UNext(3, 1)
    spec = O.unext_param_spec(3, 1)
    sd = m.state_dict()
    assert [k for k, _ in spec] == list(sd.keys())
    for k, shape in spec:
        assert tuple(sd[k].shape) == tuple(shape), k
    n = sum(p.numel() for p in m.parameters())
    assert n == 1471921  # UNeXt's published 1.47 M parameters


def test_oracle_shift_is_an_index_shift():
    g = torch.Generator().manual_seed(0)
    for C in (160, 128, 256, 8):
        x = torch.randn(2, C, 6, 7, generator=g, dtype=torch.float64)
        chunk = -(-C // 5)
        for axis in (2, 3):
            y = O._shift(x, axis)
            ref = torch.zeros_like(x)
            for c in range(C):
                s = c // chunk - 2
                if axis == 2:
                    for h in range(6):
                        if 0 <= h - s < 6:
                            ref[:, c, h] = x[:, c, h - s]
                else:
                    for w in range(7):
                        if 0 <= w - s < 7:
                            ref[:, c, :, w] = x[:, c, :, w - s]
            assert torch.equal(y, ref)


def _oracle_unext(sd, x, mask, dtype):
    sdo = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
    params = {k: v.requires_grad_(True) for k, v in sdo.items() if not k.endswith(BUF)}
    out = O.unext_forward(sdo, x.to(dtype), training=True)
    loss = O.dice_bce_loss(out, mask.to(dtype))
    loss.backward()
    d = {"out": out.detach(), "loss": loss.detach().reshape(1)}
    for k, p in params.items():
        d["grad:" + k] = p.grad if p.grad is not None else torch.zeros_like(p)
    for k, v in sdo.items():
        if k.endswith(("running_mean", "running_var")):
            d["buf:" + k] = v.detach()
    return d


@pytest.mark.gpu
def test_unext_ops_match_torch():
    from accunet import unext as U
    dev = "cuda"
    g = torch.Generator().manual_seed(1)
    # LayerNorm over channels, fwd + bwd
    x = torch.randn(2, 5, 7, 160, generator=g)
    ln = torch.nn.LayerNorm(160)
    ln.weight.data = torch.rand(160, generator=g) + 0.5
    ln.bias.data = torch.randn(160, generator=g) * 0.1
    lnd = ln.double()
    xd = x.double().requires_grad_(True)
    ref = lnd(xd)
    dy = torch.randn(ref.shape, generator=g)
    ref.backward(dy.double())
    lng = torch.nn.LayerNorm(160).to(dev)
    lng.load_state_dict({k: v.float() for k, v in lnd.state_dict().items()})
    xg = x.to(dev).requires_grad_(True)
    y = U.layernorm(xg, lng)
    y.backward(dy.to(dev))
    assert (y.detach().cpu().double() - ref.detach()).abs().max() < 1e-5
    assert (xg.grad.cpu().double() - xd.grad).abs().max() < 1e-4
    assert (lng.weight.grad.cpu().double() - lnd.weight.grad).abs().max() < 1e-4
    assert (lng.bias.grad.cpu().double() - lnd.bias.grad).abs().max() < 1e-4
    # GELU
    x = torch.randn(3, 4, 4, 32, generator=g) * 3
    xd = x.double().requires_grad_(True)
    ref = F.gelu(xd)
    ref.backward(dy[..., :32].reshape(-1)[: x.numel()].reshape(x.shape).double())
    xg = x.to(dev).requires_grad_(True)
    y = U.gelu(xg)
    y.backward(dy[..., :32].reshape(-1)[: x.numel()].reshape(x.shape).to(dev))
    assert (y.detach().cpu().double() - ref.detach()).abs().max() < 1e-5
    assert (xg.grad.cpu().double() - xd.grad).abs().max() < 1e-5
    # token shift (NHWC) vs the oracle's pad/chunk/roll/narrow (NCHW)
    for C in (160, 256, 128):
        x = torch.randn(2, 6, 9, C, generator=g)
        for axis, oaxis in ((0, 2), (1, 3)):
            ref = O._shift(x.permute(0, 3, 1, 2), oaxis).permute(0, 2, 3, 1)
            xg = x.to(dev).requires_grad_(True)
            y = U.token_shift(xg, axis)
            assert torch.equal(y.detach().cpu(), ref)
            d = torch.randn(y.shape, generator=g)
            y.backward(d.to(dev))
            xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
            O._shift(xr, oaxis).backward(d.permute(0, 3, 1, 2))
            assert torch.equal(xg.grad.cpu(), xr.grad.permute(0, 2, 3, 1))
    # relu(bilinear x2) + skip
    for (H, W) in ((7, 7), (4, 6), (1, 3)):
        x = torch.randn(2, H, W, 16, generator=g)
        sk = torch.randn(2, 2 * H, 2 * W, 16, generator=g)
        xd = x.double().permute(0, 3, 1, 2).requires_grad_(True)
        ref = F.relu(F.interpolate(xd, scale_factor=(2, 2), mode="bilinear")).permute(0, 2, 3, 1) \
            + sk.double()
        d = torch.randn(ref.shape, generator=g)
        ref.backward(d.double())
        xg = x.to(dev).requires_grad_(True)
        y = U.up2_relu_add(xg, sk.to(dev))
        y.backward(d.to(dev))
        assert (y.detach().cpu().double() - ref.detach()).abs().max() < 1e-5
        assert (xg.grad.cpu().double() - xd.grad.permute(0, 2, 3, 1)).abs().max() < 1e-5
    # stride-2 pick
    x = torch.randn(2, 8, 6, 4, generator=g).to(dev).requires_grad_(True)
    y = U.subsample2(x)
    assert torch.equal(y.detach(), x.detach()[:, ::2, ::2])
    y.backward(torch.ones_like(y))
    ref = torch.zeros(x.shape)
    ref[:, ::2, ::2] = 1
    assert torch.equal(x.grad.cpu(), ref)


@pytest.mark.gpu
def test_unext_eval_matches_reference_golden():
    """The HIP UNeXt in eval mode against the reference module's own fp32 output
    (tests/golden/unext.npz) at 2x3x64x64 and 1x3x224x224, within 1e-4 (the north-star
    bound on probabilities)."""
    from accunet.unext import UNext
    g = np.load(os.path.join(HERE, "golden", "unext.npz"))
    sd = O.det_state_dict(O.unext_param_spec(3, 1), seed=5)
    for name, shape in (("s64", (2, 3, 64, 64)), ("s224", (1, 3, 224, 224))):
        m = UNext(3, 1, img_size=shape[-1])
        m.load_state_dict(sd)
        m = m.cuda().eval()
        with torch.no_grad():
            out = m(O.det_input(shape, f"unext-x-{name}").cuda())
        d = np.abs(out.double().cpu().numpy() - g[f"out_eval_{name}"]).max()
        assert d < 1e-4, (name, d)


@pytest.mark.gpu
def test_unext_train_step_matches_oracle():
    from accunet.loss import WeightedDiceBCE
    from accunet.unext import UNext
    B, S = 2, 64
    sd = O.det_state_dict(O.unext_param_spec(3, 1), seed=0)
    x = O.det_input((B, 3, S, S), "unext-x")
    mask = O.det_mask((B, 1, S, S), "unext-mask", p=0.4)
    r64 = _oracle_unext(sd, x, mask, torch.float64)
    r32 = _oracle_unext(sd, x, mask, torch.float32)
    g = torch.Generator().manual_seed(5)

    def jit(t):
        if not t.is_floating_point():
            return t.clone()
        u = torch.rand(t.shape, generator=g, dtype=torch.float64) * 2 - 1
        return (t.double() * (1 + u * 2.0 ** -24)).float()
    extra = [_oracle_unext({k: (v.clone() if k.endswith(BUF) else jit(v)) for k, v in sd.items()},
                           jit(x), mask, torch.float32) for _ in range(2)]
    m = UNext(3, 1)
    m.load_state_dict(sd)
    m = m.cuda().train()
    out = m(x.cuda())
    loss = WeightedDiceBCE(0.5, 0.5)(out, mask.cuda())
    loss.backward()
    hip = {"out": out.detach().cpu(), "loss": loss.detach().cpu().reshape(1)}
    for k, p in m.named_parameters():
        hip["grad:" + k] = p.grad.detach().cpu() if p.grad is not None else torch.zeros_like(p).cpu()
    for k, v in m.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            hip["buf:" + k] = v.detach().cpu()
    med = float(np.median([r64[k].abs().mean().item() for k in r64 if k.startswith("grad:")]))
    # conv biases feeding a BatchNorm have an (analytically) zero gradient: only fp noise
    bn_fed = {f"grad:{n}.bias": 1e-6 * med for n in ("encoder1", "encoder2", "encoder3",
                                                      "decoder1", "decoder2", "decoder3",
                                                      "decoder4")}
    rows = PU.compare_vs_reference_fp32(hip, r64, r32, factor=4.0, rel_floor=1e-4,
                                        abs_floor=bn_fed, ref32_extra=extra)
    bad = [r for r in rows if not r[4]]
    assert not bad, bad[:8]
    assert abs(float(hip["loss"]) - float(r64["loss"])) < 1e-5


@pytest.mark.gpu
def test_unext_full_size_config_properties():
    """BASELINE configs[4] at full size (32 x 3 x 224 x 224), where the fp64 oracle is
    too slow: bit-identical repeated steps, finite gradients, probabilities in [0, 1],
    the loss kernel equal to WeightedDiceBCE recomputed in fp64 from the HIP output,
    and three Adam steps on one batch lower the loss."""
    from accunet.loss import WeightedDiceBCE
    from accunet.train import TrainStep
    from accunet.unext import UNext
    torch.manual_seed(0)
    m = UNext(3, 1).cuda().train()
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(5)
    x = torch.randn(32, 3, 224, 224, generator=g).cuda()
    mask = (torch.rand(32, 1, 224, 224, generator=g) < 0.3).float().cuda()
    crit = WeightedDiceBCE(0.5, 0.5)
    runs = []
    for _ in range(2):
        m.load_state_dict(sd0)
        m.zero_grad(set_to_none=True)
        out = m(x)
        loss = crit(out, mask)
        loss.backward()
        runs.append((out.detach().clone(), float(loss), [p.grad.clone() for p in m.parameters()]))
    # drop the eager autograd graph before capturing: PyTorch keeps the stream of each
    # AccumulateGrad node while a graph holding it is alive, and a capture whose
    # backward accumulates through such a node on the default stream fails
    del out, loss
    (o1, l1, g1), (o2, l2, g2) = runs
    assert torch.equal(o1, o2) and l1 == l2 and all(torch.equal(a, b) for a, b in zip(g1, g2))
    assert float(o1.min()) >= 0 and float(o1.max()) <= 1
    assert all(torch.isfinite(a).all() for a in g1)
    ref = O.dice_bce_loss(o1.double().cpu(), mask.double().cpu())
    assert abs(l1 - float(ref)) < 1e-5 * max(1.0, abs(float(ref)))
    m.load_state_dict(sd0)
    step = TrainStep(m, lr=1e-3, graph=True)
    losses = [float(step(x, mask)) for _ in range(4)]
    assert losses[-1] < losses[0], losses
