"""Host logic of ops.GradSlot (shared gradient buffers, no kernels): every
contribution order yields the same total, only the last consumer hands the buffer
to autograd, pass-through gradients are read (never written), and the slot resets
for the next backward. The GEMM / pool2 epilogue arithmetic it drives is covered by
the whole-model GPU tests (tests/test_model_gpu.py)."""
import itertools

import pytest
import torch

from accunet import ops


def _run(order, parts, shape):
    """Drive one backward: kinds 'gemm' (epilogue: C = new + addends), 'acc' (kernel
    accumulate flag + flush), 'give' (pass-through); returns (returned grads, slot)."""
    slot = ops.GradSlot()
    for _ in order:
        slot.register()
    outs = []
    like = torch.empty(shape, dtype=parts[0].dtype)
    for kind, g in zip(order, parts):
        if kind == "gemm":
            buf, adds = slot.gemm_target(shape, like)
            total = g.clone()
            for t in adds:
                total += t
            buf.copy_(total)
        elif kind == "acc":
            buf, acc = slot.acc_target(shape, like)
            if acc:
                buf += g
            else:
                buf.copy_(g)
            slot.flush()
        else:
            slot.give(g)
        outs.append(slot.done())
    return outs, slot


@pytest.mark.parametrize("order", sorted(set(itertools.permutations(["gemm", "acc", "give", "gemm"]))))
def test_gradslot_sum_any_order(order):
    torch.manual_seed(0)
    shape = (2, 3, 4, 5)
    parts = [torch.randn(shape, dtype=torch.float64) for _ in order]
    given = [p.clone() for p in parts]
    outs, slot = _run(order, parts, shape)
    assert all(o is None for o in outs[:-1])
    torch.testing.assert_close(outs[-1], sum(parts), rtol=1e-12, atol=1e-12)
    for p, g, k in zip(parts, given, order):  # pass-through gradients are never written
        if k == "give":
            assert torch.equal(p, g)
    assert not slot.live and slot.buf is None


def test_gradslot_single_give_is_returned_as_is():
    g = torch.randn(3, 4)
    outs, _ = _run(["give"], [g], (3, 4))
    assert outs[0] is g


def test_gradslot_resets_between_backwards():
    torch.manual_seed(1)
    shape = (4, 4)
    slot = ops.GradSlot()
    slot.register()
    slot.register()
    for _ in range(2):
        a, b = torch.randn(shape), torch.randn(shape)
        buf, adds = slot.gemm_target(shape, a)
        assert adds == []
        buf.copy_(a)
        assert slot.done() is None
        slot.give(b)
        out = slot.done()
        torch.testing.assert_close(out, a + b)


def test_gradslot_consumer_without_gradient():
    """a consumer whose output went unused still counts (done() with no contribution)"""
    shape = (2, 2)
    slot = ops.GradSlot()
    for _ in range(3):
        slot.register()
    g = torch.ones(shape)
    assert slot.done() is None
    slot.give(g)
    assert slot.done() is None
    assert slot.done() is g


def test_gradslot_folds_extra_addends():
    """more than three pending contributions: the epilogue's three addend slots suffice"""
    torch.manual_seed(2)
    shape = (3, 3)
    slot = ops.GradSlot()
    parts = [torch.randn(shape, dtype=torch.float64) for _ in range(5)]
    for _ in parts:
        slot.register()
    for p in parts[:4]:
        slot.give(p.clone())
        assert slot.done() is None
    buf, adds = slot.gemm_target(shape, parts[0])
    assert len(adds) <= 3
    buf.copy_(parts[4] + sum(adds))
    torch.testing.assert_close(slot.done(), sum(parts), rtol=1e-12, atol=1e-12)


def test_gradslot_fold_never_writes_given_tensors():
    """give() promises its tensors are only read: with more than three contributions
    the fold goes into a tensor the slot owns, never into a given (autograd-owned)
    gradient such as a residual add's incoming dy. The tensors are passed without
    cloning, and must be unchanged afterwards."""
    torch.manual_seed(3)
    shape = (3, 3)
    slot = ops.GradSlot()
    parts = [torch.randn(shape, dtype=torch.float64) for _ in range(5)]
    keep = [p.clone() for p in parts]
    for _ in parts:
        slot.register()
    for p in parts[:4]:
        slot.give(p)
        assert slot.done() is None
    buf, adds = slot.gemm_target(shape, parts[0])
    assert len(adds) <= 3
    buf.copy_(parts[4] + sum(adds))
    torch.testing.assert_close(slot.done(), sum(keep), rtol=1e-12, atol=1e-12)
    for p, k in zip(parts, keep):
        assert torch.equal(p, k)
