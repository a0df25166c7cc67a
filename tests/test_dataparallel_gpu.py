"""The reference's evaluation wrapping (Experiments/test_model.py:220-224):

    model = ACC_UNet(n_channels=..., n_classes=..., n_filts=...)
    if torch.cuda.device_count() > 1:
        model = nn.DataParallel(model, device_ids=[0, 1, 2, 3])
    model.load_state_dict(checkpoint['state_dict'])

On a multi-GPU node nn.DataParallel replicates the module onto every device
(torch.nn.parallel.replicate: parameters broadcast as non-leaf tensors, buffers
copied) and runs one replica per input chunk. The drop-in must compute on a replica
exactly what it computes bare, and route gradients through the broadcast back to the
original parameters. The test box has one GPU, so device_ids=[0] (DataParallel then
calls the module itself) and an explicit replicate() onto device 0 (the replica path
each of the reference's four devices takes).
"""
import os
import sys

import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from parity_util import O  # noqa: E402
from nets.ACC_UNet import ACC_UNet  # noqa: E402  (the reference's import path)
from accunet.loss import WeightedDiceBCE  # noqa: E402

DEV = "cuda"


def _model(sd):
    m = ACC_UNet(n_channels=3, n_classes=1, n_filts=8)
    m.load_state_dict(sd)
    return m.to(DEV)


def _data():
    x = O.det_input((2, 3, 32, 32), "dp-x").to(DEV)
    mask = O.det_mask((2, 1, 32, 32), "dp-mask", p=0.4).to(DEV)
    return x, mask


def test_dataparallel_wrapping_matches_bare_module():
    sd = O.det_state_dict(O.param_spec("script", 3, 1, 8), seed=0)
    x, _ = _data()
    for train in (False, True):
        bare = _model(sd).train(train)
        wrapped = nn.DataParallel(_model(sd), device_ids=[0]).train(train)
        # the checkpoint round trip of test_model.py: a DataParallel state_dict has
        # "module."-prefixed keys and loads back into the wrapper
        wrapped.load_state_dict({"module." + k: v for k, v in sd.items()})
        with torch.no_grad():
            y0 = bare(x)
            y1 = wrapped(x)
        torch.cuda.synchronize()
        assert torch.equal(y0, y1), (train, float((y0 - y1).abs().max()))
        if train:  # running statistics updated the same way
            for (k, a), b in zip(bare.state_dict().items(), wrapped.module.state_dict().values()):
                assert torch.equal(a, b), k


def test_replica_forward_backward_matches_bare_module():
    """torch.nn.parallel.replicate (what nn.DataParallel does per device): the replica's
    train forward + WeightedDiceBCE + backward gives the bare module's output, loss and
    every parameter gradient bit for bit, the gradients arriving through the broadcast
    on the ORIGINAL parameters."""
    sd = O.det_state_dict(O.param_spec("script", 3, 1, 8), seed=0)
    x, mask = _data()
    crit = WeightedDiceBCE(0.5, 0.5)
    bare = _model(sd).train()
    y0 = bare(x)
    l0 = crit(y0, mask)
    l0.backward()
    src = _model(sd).train()
    rep = nn.parallel.replicate(src, [0])[0]
    assert all(not p.is_leaf for p in rep.parameters())  # broadcast copies, not the Parameters
    y1 = rep(x)
    l1 = crit(y1, mask)
    l1.backward()
    torch.cuda.synchronize()
    assert torch.equal(y0.detach(), y1.detach())
    assert float(l0) == float(l1)
    n = 0
    for (k, p0), p1 in zip(bare.named_parameters(), src.parameters()):
        if p0.grad is None:
            assert p1.grad is None, k
            continue
        assert p1.grad is not None, k
        assert torch.equal(p0.grad, p1.grad), (k, float((p0.grad - p1.grad).abs().max()))
        n += 1
    assert n > 100
