"""Fused ACC-UNet operators as autograd Functions over the HIP C ABI.

Activations are NHWC tensors [B, H, W, C], stored fp32 or bf16 (the model's
activation dtype; every op keeps the dtype of its input, kern.* passes it to the
kernels as ACC_F32 / ACC_BF16); parameters, their gradients and all BatchNorm / SE
state stay fp32, statistics fp64. A BatchNorm2d(+LeakyReLU) whose
statistics are known but which has not been applied yet travels as a `Pending`
(tensor z + the BatchNorm module + the partial statistics its producer's epilogue
wrote); the op that consumes it finalises the statistics (running-stat update
happens there, exactly once per forward, as in torch) and applies the
normalisation in registers while loading. The reference applies every
BatchNorm as a separate ATen pass (ACC_UNet/ACC_UNet.py, e.g. :269-284).

Every forward / backward below calls only `kern.*` (libaccunet_hip.so); torch is
used for allocation, views and autograd bookkeeping.
"""
from __future__ import annotations

import contextlib
import ctypes

import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from . import _lib, kern
from . import profile as _prof
from ._lib import (ACT_LRELU, ACT_NONE, AMODE_COL, AMODE_SHIFT3, BMODE_NN, BMODE_NN_SHIFT3,
                   PRO_AFFINE, PRO_AFFINE_LRELU, PRO_NONE)

__all__ = ["Pending", "GradSlot", "pw_conv", "dw_conv", "hanc_layer", "bn_act_add", "se", "conv3x3",
           "conv_transpose2x2", "conv_transpose2x2_cat", "pool2", "cat_channels", "head", "wmerge", "group_relayout",
           "to_nhwc", "weighted_dice_bce"]


def _f32(shape, like):
    """fp32 tensor (parameter-shaped / state / model output) on like's device."""
    return torch.empty(shape, dtype=torch.float32, device=like.device)


def _act(shape, like):
    """activation-shaped tensor with like's storage dtype (fp32 or bf16)."""
    return torch.empty(shape, dtype=like.dtype, device=like.device)


def _stats(shape, like):
    """fp64 partial-statistics block [rows, 2, C] (see include/accunet.h)."""
    return torch.empty(shape, dtype=torch.float64, device=like.device)


def _flat_off(t: torch.Tensor, off: int) -> torch.Tensor:
    """1-D view of t starting `off` elements in (pointer offset for kernels)."""
    f = t.view(-1)
    return f.narrow(0, off, f.numel() - off)


# --------------------------------------------------------------------------
# Weight gradients on a side stream
# --------------------------------------------------------------------------
# ACCUNET_WGRAD_STREAM=0 keeps every backward kernel on one stream (A/B runs).
_WGRAD_STREAM = os.environ.get("ACCUNET_WGRAD_STREAM", "1") != "0"
# fork only weight gradients estimated to take at least this many microseconds (each
# fork / join is a cross-queue graph edge with its own latency; 0 = fork every one)
_FORK_MIN_US = float(os.environ.get("ACCUNET_WGRAD_FORK_MIN_US", "0"))
_SIDE_STREAMS = {}
FORK_COUNTS = [0, 0]  # weight gradients kept on the main stream / forked (diagnostics)
FORK_LOG = None  # a list: the estimated side-branch microseconds of every fork decision


def set_wgrad_stream(on: bool) -> bool:
    """Enable / disable the side-stream weight gradients; returns the previous setting."""
    global _WGRAD_STREAM
    prev = _WGRAD_STREAM
    _WGRAD_STREAM = bool(on)
    return prev


def set_wgrad_fork_min_us(us: float) -> float:
    """Fork only weight gradients estimated at >= `us` microseconds (0 = fork every one;
    the default comes from ACCUNET_WGRAD_FORK_MIN_US); returns the previous cut."""
    global _FORK_MIN_US
    prev = _FORK_MIN_US
    _FORK_MIN_US = float(us)
    return prev


class _WgradFork:
    """Runs a backward's weight-gradient GEMMs on a side stream, concurrently with its
    data-gradient chain (data-gradient GEMM, BatchNorm backward, column sums): both
    only read dZ and the saved inputs, and write disjoint buffers. Under graph
    capture the fork / join become graph edges, so the replayed backward has two
    branches per layer.

    Memory safety: the side stream first waits for the main stream; `join()` (main
    waits for side) runs before the backward returns, so every tensor the side stream
    read or wrote is freed -- or handed to autograd -- after the join in main-stream
    order, and the caching allocator never hands out a block the side stream still
    uses. The one-launch statistics reductions (reduce_finish) enqueued on the side
    stream use ticket bank 1 (registered per stream in the library when the stream is
    created), every other stream bank 0, so concurrent reductions never share a ticket
    counter, whichever thread enqueues them."""

    def __init__(self, like: torch.Tensor, flops: float = 0.0, nbytes: float = 0.0):
        # (flops, nbytes): the side branch's work, for the ACCUNET_WGRAD_FORK_MIN_US cut
        # (estimated at 100 TFLOP/s and 5 TB/s)
        est_us = max(flops / 1e8, nbytes / 5e6)
        self.on = _WGRAD_STREAM and like.is_cuda and est_us >= _FORK_MIN_US
        if _WGRAD_STREAM and like.is_cuda:
            FORK_COUNTS[int(self.on)] += 1
            if FORK_LOG is not None:
                FORK_LOG.append(est_us)
        if not self.on:
            return
        self.main = torch.cuda.current_stream(like.device)
        side = _SIDE_STREAMS.get(like.device.index)
        if side is None:
            side = _SIDE_STREAMS[like.device.index] = torch.cuda.Stream(device=like.device)
            kern.stream_ticket_bank(side, 1)
        self.side = side
        side.wait_stream(self.main)

    def __enter__(self):
        if self.on:
            self._ctx = torch.cuda.stream(self.side)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.on:
            self._ctx.__exit__(*exc)
        return False

    def join(self):
        if self.on:
            self.main.wait_stream(self.side)


# --------------------------------------------------------------------------
# Pending BatchNorm(+act)
# --------------------------------------------------------------------------
class Pending:
    """value = act(bn(z)); bn None -> value = z (already materialised).

    bslot: optional _BiasSlot of the convolution that produced z. The consumer's
    BatchNorm backward fills it with sum_p dz, which is that convolution's bias
    gradient (z feeds only this BatchNorm), so the producer's backward needs no
    separate column-sum pass over dz."""

    __slots__ = ("z", "bn", "act", "part", "rows", "bslot")

    def __init__(self, z: torch.Tensor, bn=None, act: int = ACT_NONE, part=None, rows: int = 0,
                 bslot=None):
        self.z = z
        self.bn = bn
        self.act = act
        self.part = part
        self.rows = rows
        self.bslot = bslot


class _BiasSlot:
    """Bias gradient of a producer convolution, written by its consumer's backward."""

    __slots__ = ("t",)

    def __init__(self):
        self.t = None


def _bias_slot(bias, consumer_bn):
    return _BiasSlot() if (bias is not None and consumer_bn is not None) else None


def _take_bias_grad(slot):
    """the consumer-computed bias gradient, or None (then the producer sums dZ itself)"""
    if slot is None or slot.t is None:
        return None
    t, slot.t = slot.t, None
    return t


class GradSlot:
    """One shared gradient buffer for an activation that several ops consume (MLFC's
    level inputs and their pooled copies, ACC_UNet.py:427-525; the ResPath chain and
    the encoder skips, :290-328, :612-620). Each consumer registers in its forward.
    In backward the consumers' contributions meet in one buffer: a GEMM data gradient
    writes it and folds the contributions that arrived before it in as epilogue
    addends (the buffer itself and any pass-through gradients, read, not copied),
    pool2 accumulates with its kernel flag, a residual add hands its incoming
    gradient over untouched (`give`). The last consumer to finish returns the buffer
    to autograd and the others return None, so autograd never runs an elementwise
    add to sum them. Contributions arrive in autograd's execution order, which a
    captured graph fixes, so the sum is deterministic."""

    __slots__ = ("n", "left", "buf", "pend", "live")

    def __init__(self):
        self.n = 0
        self.left = 0
        self.buf = None
        self.pend = []
        self.live = False

    def register(self):
        self.n += 1
        return self

    def _begin(self):
        if not self.live:
            self.live = True
            self.left = self.n
            self.buf = None
            self.pend = []

    def give(self, g):
        """contribute g as it is (read later as an addend, never written)."""
        self._begin()
        self.pend.append(g)

    def gemm_target(self, shape, like):
        """(buffer, addends) for a GEMM epilogue: C = A*B + sum(addends), in place."""
        self._begin()
        adds = ([self.buf] if self.buf is not None else []) + self.pend
        if self.buf is None:
            self.buf = torch.empty(shape, dtype=like.dtype, device=like.device)
        self.pend = []
        if len(adds) > 3:  # the epilogue takes three addends; fold the rest first
            # into a tensor this slot owns: the shared buffer when it already holds a
            # contribution, else a copy -- give() tensors are read, never written
            acc = adds[0] if adds[0] is self.buf else adds[0].clone()
            for t in adds[3:]:
                acc.add_(t)
            adds = [acc] + adds[1:3]
        return self.buf, adds

    def acc_target(self, shape, like):
        """(buffer, accumulate) for a kernel with an accumulate flag; call flush() after."""
        self._begin()
        if self.buf is None:
            self.buf = torch.empty(shape, dtype=like.dtype, device=like.device)
            return self.buf, False
        return self.buf, True

    def flush(self):
        for t in self.pend:
            self.buf.add_(t)
        self.pend = []

    def done(self):
        """a consumer finished (contributed or not): the gradient for the last one."""
        self._begin()
        self.left -= 1
        if self.left > 0:
            return None
        if self.buf is None and self.pend:
            self.buf = self.pend.pop(0) if len(self.pend) == 1 else self.pend.pop(0).clone()
        if self.pend:
            self.flush()
        b, self.buf, self.live = self.buf, None, False
        return b


_SLOTS_ON = os.environ.get("ACCUNET_GRADSLOT", "1") != "0"  # 0: autograd sums (A/B runs)


def _slot_reg(slot):
    if slot is None or not _SLOTS_ON or not torch.is_grad_enabled():
        return None
    return slot.register()


# --------------------------------------------------------------------------
# Forward-layout weight copies made ahead of time (graph mode)
# --------------------------------------------------------------------------
_PREP = None  # {(weight data_ptr, tag): tensor} while a WeightPrep is active


def _prepared(weight, tag):
    """the forward-layout copy of `weight` made by the active WeightPrep, or None (then
    the op makes it itself)"""
    if _PREP is None:
        return None
    return _PREP.get((weight.data_ptr(), tag))


class WeightPrep:
    """Every forward-layout weight copy of a model -- HANCLayer's grouped columns
    (ACC_UNet.py:96-106,138), the MLFC merge de-interleave (:492), the ResPath 3x3 and
    its flipped data-gradient form (:317-318), the ConvTranspose2d [ci][tap][co] form
    (:578-590) -- made by ONE launch (accunet_relayout_batch) into persistent buffers.

    The graph-mode TrainStep runs it before each replay and captures its graph inside
    `active()`, so the captured ops read these buffers instead of launching ~54 small
    relayouts per step. Outside `active()` every op makes its own copy, so an eager
    forward (validation, tests) never reads a copy older than the weights."""

    def __init__(self, model):
        from torch import nn
        from .model import HANCLayer, MLFC, MLFC_Lite, ResPath
        items, bufs, keep = [], {}, []

        def add(w, tag, out_shape, kind, **kw):
            key = (w.data_ptr(), tag)
            if key in bufs:
                return
            out = torch.empty(out_shape, dtype=torch.float32, device=w.device)
            it = _lib.AccRelayout()
            it.inp, it.out = w.data_ptr(), out.data_ptr()
            it.total, it.kind = out.numel(), kind
            if kind == 0:
                for a in range(4):
                    it.d[a], it.s[a] = kw["d"][a], kw["s"][a]
                    it.flip[a] = kw.get("flip", (0, 0, 0, 0))[a]
            else:
                it.N, it.C, it.J = kw["N"], kw["C"], kw["J"]
                for j in range(8):
                    it.order[j] = kw["order"][j] if j < kw["J"] else j
            items.append(it)
            bufs[key] = out
            keep.append(w)

        for m in model.modules():
            if isinstance(m, HANCLayer):
                w = m.cnv.weight
                N, K = w.shape[0], w.shape[1]
                J = 2 * m.k - 1
                add(w, "hanc", (N, K), 1, N=N, C=K // J, J=J, order=_HANC_ORDER[m.k])
            elif isinstance(m, MLFC) and not isinstance(m, MLFC_Lite):
                for name, ch in m.named_children():
                    if name.startswith("cnv_mrg"):
                        for blk in ch:
                            w = blk.conv1.weight
                            f = w.shape[0]
                            add(w, "grp", (f, 2 * f), 1, N=f, C=f, J=2, order=(0, 1))
            elif isinstance(m, ResPath):
                for conv in m.convs:
                    w = conv.weight
                    Co, Ci = w.shape[0], w.shape[1]
                    add(w, "c3", (Co, 9 * Ci), 0, d=(Co, 3, 3, Ci), s=(9 * Ci, 3, 1, 9))
                    add(w, "c3f", (Ci, 9 * Co), 0, d=(Ci, 3, 3, Co), s=(9, 3, 1, 9 * Ci),
                        flip=(0, 1, 1, 0))
            elif isinstance(m, nn.ConvTranspose2d) and tuple(m.kernel_size) == (2, 2):
                w = m.weight
                Ci, Co = w.shape[0], w.shape[1]
                add(w, "ct", (Ci, 4 * Co), 0, d=(Ci, 2, 2, Co), s=(4 * Co, 2, 1, 4))
        blk = 0
        for it in items:
            it.blk0 = blk
            blk += kern.relayout_blocks(it.total)
        self.n, self.nblocks = len(items), blk
        self.bufs = bufs
        self._weights = keep
        self._items = items
        if items:
            raw = bytes((_lib.AccRelayout * len(items))(*items))
            dev = keep[0].device
            self.table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)

    def run(self):
        """(re)make every copy from the current weights, on the current stream"""
        if self.n:
            kern.relayout_batch(self.table, self.n, self.nblocks)

    @contextlib.contextmanager
    def active(self):
        global _PREP
        prev, _PREP = _PREP, self.bufs
        try:
            yield self
        finally:
            _PREP = prev


_DEFER = None  # DeferredRelayouts collecting the backward's inverse weight relayouts


class DeferredRelayouts:
    """The backward's inverse weight relayouts -- HANCLayer / MLFC-merge weight
    gradients from the grouped GEMM columns back to the reference's interleave, the
    ResPath 3x3 and ConvTranspose2d weight gradients back to the torch layout -- taken
    out of the per-layer backward and made by batched accunet_relayout_batch launches
    in a captured backward (graph-mode TrainStep). Inside `active()` the backward ops
    append items instead of launching; each `flush()` captures one launch over the items
    added since the previous flush, reading its own segment of a preallocated item
    table, and `upload()` fills every segment after the capture (the addresses are the
    graph pool's, fixed for every replay). At world 1 there is one flush, after
    loss.backward() (every side-stream weight-gradient fork has joined the main stream by
    then). With data parallelism a gradient bucket must hold final values when it is
    packed for its all-reduce, so the bucket's seal flushes first (train._GraphBuckets):
    one launch per sealed bucket instead of one per layer (the ops join their forks
    before they return, so every pending item's source is final at a seal)."""

    CAP = 128

    def __init__(self, device, cap=None):
        self.cap = cap or self.CAP
        self.items, self.keep = [], []
        self.table = torch.zeros(self.cap * ctypes.sizeof(_lib.AccRelayout), dtype=torch.uint8,
                                 device=device)
        self.done = 0        # items already captured by a flush
        self.segments = []   # (byte offset in the table, item bytes) per flush
        self.launches = 0

    def full(self):
        return len(self.items) >= self.cap

    def _add(self, src, dst, kind, total, **kw):
        it = _lib.AccRelayout()
        it.inp, it.out = src.data_ptr(), dst.data_ptr()
        it.total, it.kind = int(total), kind
        if kind in (3, 4):
            it.scale = kw.get("scale", 1.0)
        elif kind == 0:
            for a in range(4):
                it.d[a], it.s[a] = kw["d"][a], kw["s"][a]
                it.flip[a] = 0
        else:
            it.N, it.C, it.J = kw["N"], kw["C"], kw["J"]
            for j in range(8):
                it.order[j] = kw["order"][j] if j < kw["J"] else j
        self.items.append(it)
        # the source stays alive here; the destination is the gradient autograd hands to
        # the parameter: an extra reference would make AccumulateGrad clone it (copy the
        # still-unfilled buffer) instead of taking it, so only its address is kept, and
        # TrainStep checks after the capture that every one became a parameter's .grad
        self.keep.append(src)

    def permute(self, src, dst, d, s):
        self._add(src, dst, 0, dst.numel(), d=d, s=s)

    def group_inverse(self, src, dst, N, C, J, order):
        self._add(src, dst, 2, N * J * C, N=N, C=C, J=J, order=order)

    def copy(self, src, dst, scale=1.0):
        """flat copy of a contiguous fp32 tensor times `scale` into dst (fp32, or bf16
        rounded to nearest even): kinds 3 / 4, the data-parallel bucket packing"""
        if src.dtype != torch.float32 or dst.numel() != src.numel():
            raise ValueError("copy: fp32 source of dst's size")
        self._add(src, dst, 4 if dst.dtype == torch.bfloat16 else 3, src.numel(), scale=scale)

    def flush(self):
        """one launch for the items added since the last flush (none: no launch)"""
        new = self.items[self.done:]
        if not new:
            return
        blk = 0
        for it in new:
            it.blk0 = blk
            blk += kern.relayout_blocks(it.total)
        sz = ctypes.sizeof(_lib.AccRelayout)
        off = self.done * sz
        raw = bytes((_lib.AccRelayout * len(new))(*new))
        self.segments.append((off, raw))
        kern.relayout_batch(self.table[off:], len(new), blk)
        self.done = len(self.items)
        self.launches += 1

    def destinations(self):
        return [int(it.out) for it in self.items]

    def upload(self):
        for off, raw in self.segments:
            self.table[off:off + len(raw)].copy_(
                torch.frombuffer(bytearray(raw), dtype=torch.uint8))

    @contextlib.contextmanager
    def active(self):
        global _DEFER
        prev, _DEFER = _DEFER, self
        try:
            yield self
        finally:
            _DEFER = prev


def _wgrad_permute(src, dst, d, s):
    """a weight gradient back to the torch layout (accunet_permute4), or deferred"""
    if _DEFER is not None and not _DEFER.full():
        _DEFER.permute(src, dst, d, s)
    else:
        kern.permute4(src, dst, d, s)


def _wgrad_group_inverse(src, dst, N, C, J, order):
    """a grouped-column weight gradient back to the reference interleave, or deferred"""
    if _DEFER is not None and not _DEFER.full():
        _DEFER.group_inverse(src, dst, N, C, J, order)
    else:
        kern.group_relayout(src, dst, N, C, J, order, inverse=True)


def as_pending(x) -> Pending:
    return x if isinstance(x, Pending) else Pending(x)


@dataclass
class _Pro:
    """Finalised BatchNorm prologue for one consumer (non-tensor context)."""
    active: bool
    st: Optional[torch.Tensor] = None   # [4, C] mean, rstd, scale, shift
    act: int = ACT_NONE
    training: bool = False
    bslot: object = None  # the producer's _BiasSlot (filled with sum_p dz in backward)


def _finalize(p: Pending) -> _Pro:
    if p.bn is None:
        return _Pro(False)
    bn = p.bn
    z = p.z
    C = z.shape[-1]
    P = z.numel() // C
    training = bn.training or not bn.track_running_stats
    st = _f32((4, C), z)
    if training and p.part is None:
        raise RuntimeError("pending BatchNorm in training mode without producer statistics")
    mom = bn.momentum if bn.momentum is not None else 0.1
    kern.bn_finalize(p.part, p.rows, C, float(P), bn.weight, bn.bias,
                     bn.running_mean if bn.track_running_stats else None,
                     bn.running_var if bn.track_running_stats else None,
                     bn.num_batches_tracked if (training and bn.track_running_stats) else None,
                     mom, bn.eps, training, st)
    return _Pro(True, st, p.act, training, p.bslot)


def _pro_mode(pro: _Pro) -> int:
    if not pro.active:
        return PRO_NONE
    return PRO_AFFINE_LRELU if pro.act == ACT_LRELU else PRO_AFFINE


def _pro_bwd(pro: _Pro, z, gamma, dA, need_z=True, need_params=True):
    """Backward of a BatchNorm(+act) prologue: returns (dz, dgamma, dbeta)."""
    if not pro.active:
        return dA, None, None
    C = z.shape[-1]
    P = z.numel() // C
    dz = torch.empty_like(z)
    dg = _f32((C,), z) if need_params else None
    db = _f32((C,), z) if need_params else None
    dsum = _f32((C,), z) if pro.bslot is not None else None
    kern.bn_bwd(z, dA, pro.st, gamma, pro.act, pro.training, P, C, dz, False, dg, db, dsum)
    if dsum is not None:
        pro.bslot.t = dsum
    return dz, dg, db


def _pro_bwd_part(pro: _Pro, z, gamma, dA, part, R):
    """_pro_bwd whose reduce pass already ran in dA's producer (`part` = [R][2][C]
    partials of (sum g, sum g*(z - mean)) from a GEMM / depthwise epilogue)."""
    C = z.shape[-1]
    P = z.numel() // C
    dz = torch.empty_like(z)
    dg = _f32((C,), z)
    db = _f32((C,), z)
    dsum = _f32((C,), z) if pro.bslot is not None else None
    kern.bn_bwd_part(z, dA, pro.st, gamma, pro.act, pro.training, P, C, part, R, dz, dg, db, dsum)
    if dsum is not None:
        pro.bslot.t = dsum
    return dz, dg, db


def _bnb_part(pro: _Pro, P: int, C: int, like, rows: int):
    """partials buffer + the (z-independent part of the) epilogue request, or None."""
    if not pro.active:
        return None
    return _stats((rows, 2, C), like)


def _bn_params(p: Pending):
    if p.bn is None:
        return None, None
    return p.bn.weight, p.bn.bias


def _want_stats(consumer_bn) -> bool:
    return consumer_bn is not None and (consumer_bn.training or not consumer_bn.track_running_stats)


# --------------------------------------------------------------------------
# 1x1 convolution (multi-source, optional BN prologue on source 0, nearest-up adds)
# --------------------------------------------------------------------------
@dataclass
class _PWCfg:
    nsrc: int
    src_ch: List[int]
    pro: _Pro
    w_off: int
    w_ld: int
    N: int
    B: int
    H: int
    W: int
    ups: List[tuple] = field(default_factory=list)  # (log2f, col_off, ld)
    want_stats: bool = False
    has_bias: bool = True
    bslot: object = None
    slots: Optional[List] = None  # per source: GradSlot or None
    wslot: object = None  # GradSlot shared by the calls that write column slices of one weight


class _PWConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg: _PWCfg, weight, bias, pro_g, pro_b, *tens):
        srcs = tens[:cfg.nsrc]
        ups = tens[cfg.nsrc:]
        B, H, W, N = cfg.B, cfg.H, cfg.W, cfg.N
        P = B * H * W
        kbeg = [0]
        for c in cfg.src_ch:
            kbeg.append(kbeg[-1] + c)
        K = kbeg[-1]
        Z = _act((B, H, W, N), srcs[0])
        stats = None
        rows = 0
        if cfg.want_stats:
            rows = kern.gemm_stats_rows(P, N, K)
            stats = _stats((rows, 2, N), weight)
        pro = cfg.pro
        kern.gemm(P, N, K, a=list(srcs), lda=cfg.src_ch, kbeg=kbeg, b=weight, ldb=cfg.w_ld,
                  b_offset=cfg.w_off, c=Z, ldc=N, bias=bias if cfg.has_bias else None,
                  pro_a=_pro_mode(pro), a_scale=pro.st[2] if pro.active else None,
                  a_shift=pro.st[3] if pro.active else None, H=H, W=W,
                  ups=[(u, ld, lg, off) for u, (lg, off, ld) in zip(ups, cfg.ups)], stats=stats)
        ctx.cfg = cfg
        ctx.kbeg = kbeg
        ctx.save_for_backward(weight, pro_g, *srcs)
        ctx.up_shapes = [u.shape for u in ups]
        if stats is None:
            stats = _f32((0,), weight)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)
        ctx.rows = rows
        return Z, stats

    @staticmethod
    def backward(ctx, dZ, _dstats):
        slots = ctx.cfg.slots or [None] * ctx.cfg.nsrc
        if dZ is None:  # output unused: every input gradient is zero
            d_srcs = [sl.done() if sl is not None else None for sl in slots]
            if ctx.cfg.wslot is not None:
                raise RuntimeError("pw_conv: a weight-slice GradSlot call must reach the loss")
            return (None,) * 5 + tuple(d_srcs) + (None,) * len(ctx.up_shapes)
        cfg = ctx.cfg
        weight, pro_g, *srcs = ctx.saved_tensors
        dZ = dZ.contiguous()
        B, H, W, N = cfg.B, cfg.H, cfg.W, cfg.N
        P = B * H * W
        kbeg = ctx.kbeg
        nig = ctx.needs_input_grad  # (cfg, weight, bias, pro_g, pro_b, *srcs, *ups)
        pro = cfg.pro
        keep = []
        d_srcs = []
        dpro_g = dpro_b = None
        # weight gradient first, on the side stream (overlaps the data gradients below)
        dW = None
        cin = sum(cfg.src_ch)
        fork = _WgradFork(dZ, 2.0 * N * P * cin, float(P * (N + cin) * dZ.element_size()))
        if nig[1]:
            full = (cfg.w_off == 0 and kbeg[-1] == cfg.w_ld)
            if cfg.wslot is not None:  # the sharing calls write disjoint slices covering W
                dW, _ = cfg.wslot.acc_target(weight.shape, weight)
            else:
                dW = torch.empty_like(weight)
            with fork:
                if cfg.wslot is None and not full:
                    dW.zero_()
                for s, (x, C) in enumerate(zip(srcs, cfg.src_ch)):
                    use_pro = (s == 0 and pro.active)
                    keep.append(kern.gemm(N, C, P, a=[dZ], lda=[N], amode=AMODE_COL, b=x, ldb=C,
                                          bmode=BMODE_NN, c=dW, ldc=cfg.w_ld,
                                          c_offset=cfg.w_off + kbeg[s],
                                          pro_b=_pro_mode(pro) if use_pro else PRO_NONE,
                                          b_scale=pro.st[2] if use_pro else None,
                                          b_shift=pro.st[3] if use_pro else None,
                                          allow_split=True))
        for s, (x, C) in enumerate(zip(srcs, cfg.src_ch)):
            need = nig[5 + s] or (s == 0 and pro.active and (nig[3] or nig[4]))
            if not need:
                d_srcs.append(slots[s].done() if slots[s] is not None else None)
                continue
            if slots[s] is None:
                dA = _act((B, H, W, C), dZ)
            if s == 0 and pro.active:
                # the prologue BatchNorm's backward reduce rides in this GEMM's epilogue
                R = kern.gemm_stats_rows(P, C, N)
                part = _bnb_part(pro, P, C, dZ, R)
                keep.append(kern.gemm(P, C, N, a=[dZ], lda=[N], b=weight, ldb=cfg.w_ld,
                                      bmode=BMODE_NN, b_offset=cfg.w_off + kbeg[s], c=dA, ldc=C,
                                      stats=part, bnb=(x, pro.st, pro.act)))
                dA, dpro_g, dpro_b = _pro_bwd_part(pro, x, pro_g, dA, part, R)
            elif slots[s] is not None:
                # shared gradient buffer: the first contribution writes it, later ones
                # add in the epilogue (addend = the buffer itself, read before written)
                dA, adds = slots[s].gemm_target((B, H, W, C), dZ)
                keep.append(kern.gemm(P, C, N, a=[dZ], lda=[N], b=weight, ldb=cfg.w_ld,
                                      bmode=BMODE_NN, b_offset=cfg.w_off + kbeg[s], c=dA, ldc=C,
                                      H=H, W=W, ups=[(t, C, 0, 0) for t in adds]))
                dA = slots[s].done()
            else:
                keep.append(kern.gemm(P, C, N, a=[dZ], lda=[N], b=weight, ldb=cfg.w_ld,
                                      bmode=BMODE_NN, b_offset=cfg.w_off + kbeg[s], c=dA, ldc=C))
            d_srcs.append(dA)
        dbias = None
        if cfg.has_bias and nig[2]:
            dbias = _take_bias_grad(cfg.bslot)
            if dbias is None:
                dbias = _f32((N,), dZ)
                keep.append(kern.colsum(dZ, P, N, dbias))
        d_ups = []
        for i, ((lg, off, ld), shp) in enumerate(zip(cfg.ups, ctx.up_shapes)):
            if not nig[5 + cfg.nsrc + i]:
                d_ups.append(None)
                continue
            dG = torch.zeros(shp, dtype=dZ.dtype, device=dZ.device) if ld != N else \
                torch.empty(shp, dtype=dZ.dtype, device=dZ.device)
            kern.upsample_bwd(dZ, N, 0, _flat_off(dG, off), ld, B, H, W, N, 1 << lg)
            d_ups.append(dG)
        fork.join()
        if cfg.wslot is not None:
            dW = cfg.wslot.done()
        return (None, dW, dbias, dpro_g, dpro_b, *d_srcs, *d_ups)


def pw_conv(srcs: Sequence, weight, bias, *, w_off: int = 0, ups: Sequence = (),
            consumer_bn=None, want_stats: Optional[bool] = None,
            slots: Optional[Sequence] = None, wslot=None):
    """Z = sum_s src_s @ W[:, w_off + kbeg_s : ...]^T (+bias) (+ nearest-up adds).

    srcs[0] may be a Pending (its BatchNorm(+act) is applied in the GEMM prologue).
    ups: sequence of (G tensor [B, H>>lg, W>>lg, ld], log2 factor, column offset).
    slots: per source, a GradSlot collecting that source's gradient (or None).
    wslot: GradSlot shared by every call that uses a column slice of `weight`, when
        those slices cover it: one dW buffer, no zero fill, no autograd adds.
    Returns Pending(Z, consumer_bn, ...) carrying Z's partial statistics.
    """
    srcs = [as_pending(s) for s in srcs]
    for s in srcs[1:]:
        if s.bn is not None:
            raise ValueError("only the first source may carry a pending BatchNorm")
    if slots is not None:
        if len(slots) != len(srcs):
            raise ValueError("pw_conv: one slot (or None) per source")
        if slots[0] is not None and srcs[0].bn is not None:
            raise ValueError("pw_conv: a pending-BatchNorm source cannot share a GradSlot")
        slots = [_slot_reg(sl) for sl in slots]
        if all(sl is None for sl in slots):
            slots = None
    pro = _finalize(srcs[0])
    z0 = srcs[0].z
    B, H, W = z0.shape[:3]
    w2 = weight.reshape(weight.shape[0], -1)
    N, w_ld = w2.shape
    if want_stats is None:
        want_stats = _want_stats(consumer_bn)
    cfg = _PWCfg(nsrc=len(srcs), src_ch=[s.z.shape[-1] for s in srcs], pro=pro, w_off=w_off,
                 w_ld=w_ld, N=N, B=B, H=H, W=W,
                 ups=[(lg, off, g.shape[-1]) for g, lg, off in ups], want_stats=want_stats,
                 has_bias=bias is not None, bslot=_bias_slot(bias, consumer_bn), slots=slots,
                 wslot=_slot_reg(wslot) if weight.requires_grad else None)
    pg, pb = _bn_params(srcs[0])
    Z, stats = _PWConvFn.apply(cfg, w2, bias, pg, pb, *[s.z for s in srcs],
                               *[g for g, _, _ in ups])
    return Pending(Z, consumer_bn, ACT_LRELU, stats if want_stats else None,
                   stats.shape[0] if want_stats else 0, bslot=cfg.bslot)


# --------------------------------------------------------------------------
# depthwise 3x3 (HANCBlock.conv2) with the norm1+LReLU prologue
# --------------------------------------------------------------------------
@dataclass
class _DWCfg:
    pro: _Pro
    B: int
    H: int
    W: int
    C: int
    want_stats: bool


class _DWConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg: _DWCfg, z, pro_g, pro_b, weight, bias):
        B, H, W, C = cfg.B, cfg.H, cfg.W, cfg.C
        Z = _act((B, H, W, C), z)
        stats = None
        if cfg.want_stats:
            stats = _stats((kern.dw3x3_rows(B, H, W, C, z), 2, C), z)
        pro = cfg.pro
        # csrc/dwconv.hip picks the LDS-tiled kernel whenever C % 32 == 0
        kname = kern.dw3x3_kernel_name(B, H, W, C, z)
        with _prof.region(f"dw3x3_fwd B{B} {H}x{W} C{C}", kernel=kname,
                          shape=f"{B}x{H}x{W}x{C}",
                          bytes_alg=2.0 * z.element_size() * B * H * W * C):
            kern.dw3x3_fwd(z, weight, bias, pro.st[2] if pro.active else None,
                           pro.st[3] if pro.active else None, pro.act, 0, Z, stats, B, H, W, C)
        ctx.cfg = cfg
        ctx.save_for_backward(z, pro_g, weight)
        if stats is None:
            stats = _f32((0,), z)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)
        return Z, stats

    @staticmethod
    def backward(ctx, dZ, _ds):
        if dZ is None:  # output unused: every input gradient is zero
            return (None,) * 6
        cfg = ctx.cfg
        z, pro_g, weight = ctx.saved_tensors
        dZ = dZ.contiguous()
        B, H, W, C = cfg.B, cfg.H, cfg.W, cfg.C
        pro = cfg.pro
        dA = torch.empty_like(z)
        dW = torch.empty_like(weight)
        db = _f32((C,), z)
        fork = _WgradFork(dZ, 18.0 * B * H * W * C, 2.0 * B * H * W * C * dZ.element_size())
        with fork:  # weight / bias gradient on the side stream (overlaps the data gradient)
            ws = kern.dw3x3_wgrad(z, dZ, pro.st[2] if pro.active else None,
                                  pro.st[3] if pro.active else None, pro.act, dW, db, B, H, W, C)
        part = R = None
        if pro.active:
            # norm1's backward reduce rides in the data-gradient kernel's epilogue
            R = kern.dw3x3_rows(B, H, W, C, dZ, bnb=True)
            part = _bnb_part(pro, B * H * W, C, z, R)
            kern.dw3x3_fwd(dZ, weight, None, None, None, ACT_NONE, 1, dA, part, B, H, W, C,
                           bnb=(z, pro.st, pro.act))
        else:
            kern.dw3x3_fwd(dZ, weight, None, None, None, ACT_NONE, 1, dA, None, B, H, W, C)
        if pro.active:
            dz, dg, dbeta = _pro_bwd_part(pro, z, pro_g, dA, part, R)
        else:
            dz, dg, dbeta = dA, None, None
        fork.join()
        del ws
        return None, dz, dg, dbeta, dW, db


def dw_conv(x, weight, bias, *, consumer_bn=None):
    x = as_pending(x)
    pro = _finalize(x)
    B, H, W, C = x.z.shape
    want = _want_stats(consumer_bn)
    cfg = _DWCfg(pro, B, H, W, C, want)
    pg, pb = _bn_params(x)
    Z, stats = _DWConvFn.apply(cfg, x.z, pg, pb, weight.reshape(C, 9), bias)
    return Pending(Z, consumer_bn, ACT_LRELU, stats if want else None,
                   kern.dw3x3_rows(B, H, W, C, x.z) if want else 0)


# --------------------------------------------------------------------------
# HANCLayer (ACC_UNet/ACC_UNet.py:77-142), restructured exactly:
#   cnv(view(cat_H[a, up2 avg2 a, up4 avg4 a, up2 max2 a, up4 max4 a]))
#   = W0 a + up2(W_{avg2,max2} [avg2 a | max2 a]) + up4(W_{avg4,max4} [avg4 a | max4 a]) + b
# --------------------------------------------------------------------------
# branch j of input channel c sits at column c*(2k-1)+j (j: 0 x, 1 avg2, 2 avg4, 3 max2,
# 4 max4 for k = 3; 0 x, 1 avg2, 2 max2 for k = 2). Relayout order groups the columns as
# [x | avg2 max2 | avg4 max4] so each GEMM reads one contiguous column block.
_HANC_ORDER = {1: [0], 2: [0, 1, 2], 3: [0, 1, 3, 2, 4]}


@dataclass
class _HancCfg:
    pro: _Pro
    k: int
    B: int
    H: int
    W: int
    C: int
    N: int
    want_stats: bool
    bslot: object = None


class _HancLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg: _HancCfg, z, pro_g, pro_b, weight, bias):
        B, H, W, C, N, k = cfg.B, cfg.H, cfg.W, cfg.C, cfg.N, cfg.k
        J = 2 * k - 1
        P = B * H * W
        pro = cfg.pro
        sc = pro.st[2] if pro.active else None
        sh = pro.st[3] if pro.active else None
        Wp = _prepared(weight, "hanc")
        if Wp is None:
            Wp = _f32((N, J * C), z)
            kern.group_relayout(weight, Wp, N, C, J, _HANC_ORDER[k])
        ups = []
        p2 = p4 = g2 = g4 = mk2 = mk4 = None
        if k >= 2:
            p2 = _act((B, H // 2, W // 2, 2 * C), z)
            p4 = _act((B, H // 4, W // 4, 2 * C), z) if k == 3 else None
            # first-max codes: the backward routes max-pool gradients with them inside
            # the x-branch data-gradient GEMM (no re-read of the activation)
            mk2 = torch.empty((B, H // 2, W // 2, C), dtype=torch.uint8, device=z.device)
            mk4 = (torch.empty((B, H // 4, W // 4, C), dtype=torch.uint8, device=z.device)
                   if k == 3 else None)
            kern.hanc_pyramid_fwd(z, sc, sh, pro.act, B, H, W, C, k, p2, p4, mk2, mk4)
            g2 = _act((B, H // 2, W // 2, N), z)
            # coarse branches: few output tiles, long K (2C) -> split-K
            keep_f = [kern.gemm(P // 4, N, 2 * C, a=[p2], lda=[2 * C], b=Wp, ldb=J * C,
                                b_offset=C, c=g2, ldc=N, allow_split=True)]
            ups.append((g2, N, 1, 0))
            if k == 3:
                g4 = _act((B, H // 4, W // 4, N), z)
                keep_f.append(kern.gemm(P // 16, N, 2 * C, a=[p4], lda=[2 * C], b=Wp,
                                        ldb=J * C, b_offset=3 * C, c=g4, ldc=N,
                                        allow_split=True))
                ups.append((g4, N, 2, 0))
        Z = _act((B, H, W, N), z)
        stats = None
        if cfg.want_stats:
            stats = _stats((kern.gemm_stats_rows(P, N, C), 2, N), z)
        with _prof.region(f"hanc_gemm P{P} N{N} K{C}", kernel="gemm_f32_kernel (HANC x-branch)",
                          shape=f"M{P} N{N} K{C}", flops=2.0 * P * N * C):
            kern.gemm(P, N, C, a=[z], lda=[C], b=Wp, ldb=J * C, c=Z, ldc=N, bias=bias,
                      pro_a=_pro_mode(pro), a_scale=sc, a_shift=sh, H=H, W=W, ups=ups,
                      stats=stats)
        ctx.cfg = cfg
        saved = [z, pro_g, Wp]
        ctx.has_p = k >= 2
        if k >= 2:
            saved += [p2, mk2]
            if k == 3:
                saved += [p4, mk4]
        ctx.save_for_backward(*saved)
        if stats is None:
            stats = _f32((0,), z)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)
        return Z, stats

    @staticmethod
    def backward(ctx, dZ, _ds):
        if dZ is None:  # output unused: every input gradient is zero
            return (None,) * 6
        cfg = ctx.cfg
        B, H, W, C, N, k = cfg.B, cfg.H, cfg.W, cfg.C, cfg.N, cfg.k
        J = 2 * k - 1
        P = B * H * W
        saved = ctx.saved_tensors
        z, pro_g, Wp = saved[:3]
        p2, mk2 = (saved[3], saved[4]) if k >= 2 else (None, None)
        p4, mk4 = (saved[5], saved[6]) if k == 3 else (None, None)
        dZ = dZ.contiguous()
        pro = cfg.pro
        sc = pro.st[2] if pro.active else None
        sh = pro.st[3] if pro.active else None
        keep = []
        dWp = _f32((N, J * C), z)
        dW = _f32((N, J * C), z)
        dP2 = dP4 = dG2 = dG4 = None
        if k >= 2:
            dG2 = _act((B, H // 2, W // 2, N), dZ)
            if k == 3:  # both pyramid sums from one read of dZ
                dG4 = _act((B, H // 4, W // 4, N), dZ)
                kern.upsample_bwd24(dZ, N, dG2, N, dG4, N, B, H, W, N)
            else:
                kern.upsample_bwd(dZ, N, 0, dG2, N, B, H, W, N, 2)
        # the three weight-gradient GEMMs on the side stream (overlap the data gradients)
        fork = _WgradFork(dZ, 2.0 * N * C * P * (1 + (1 if k >= 2 else 0) / 2 +
                                                 (1 if k == 3 else 0) / 8))
        with fork:
            if k >= 2:
                keep.append(kern.gemm(N, 2 * C, P // 4, a=[dG2], lda=[N], amode=AMODE_COL, b=p2,
                                      ldb=2 * C, bmode=BMODE_NN, c=dWp, ldc=J * C, c_offset=C,
                                      allow_split=True))
            if k == 3:
                keep.append(kern.gemm(N, 2 * C, P // 16, a=[dG4], lda=[N], amode=AMODE_COL,
                                      b=p4, ldb=2 * C, bmode=BMODE_NN, c=dWp, ldc=J * C,
                                      c_offset=3 * C, allow_split=True))
            keep.append(kern.gemm(N, C, P, a=[dZ], lda=[N], amode=AMODE_COL, b=z, ldb=C,
                                  bmode=BMODE_NN, c=dWp, ldc=J * C, c_offset=0,
                                  pro_b=_pro_mode(pro), b_scale=sc, b_shift=sh, allow_split=True))
            _wgrad_group_inverse(dWp, dW, N, C, J, _HANC_ORDER[k])
        if k >= 2:
            dP2 = _act(p2.shape, dZ)
            keep.append(kern.gemm(P // 4, 2 * C, N, a=[dG2], lda=[N], b=Wp, ldb=J * C,
                                  bmode=BMODE_NN, b_offset=C, c=dP2, ldc=2 * C))
            if k == 3:
                dP4 = _act(p4.shape, dZ)
                keep.append(kern.gemm(P // 16, 2 * C, N, a=[dG4], lda=[N], b=Wp, ldb=J * C,
                                      bmode=BMODE_NN, b_offset=3 * C, c=dP4, ldc=2 * C))
        # x branch data gradient; for k >= 2 its epilogue adds the pyramid's backward
        # (avg spread + first-max routing), so dA is written exactly once
        dA = torch.empty_like(z)
        part = R = None
        if pro.active:  # norm2's backward reduce rides in this epilogue too
            R = kern.gemm_stats_rows(P, C, N)
            part = _bnb_part(pro, P, C, z, R)
        keep.append(kern.gemm(P, C, N, a=[dZ], lda=[N], b=Wp, ldb=J * C, bmode=BMODE_NN, c=dA,
                              ldc=C, H=H, W=W,
                              pyr=(dP2, dP4, mk2, mk4) if k >= 2 else None, stats=part,
                              bnb=(z, pro.st, pro.act) if pro.active else None))
        db = _take_bias_grad(cfg.bslot)
        if db is None:
            db = _f32((N,), z)
            keep.append(kern.colsum(dZ, P, N, db))
        if pro.active:
            dz, dg, dbeta = _pro_bwd_part(pro, z, pro_g, dA, part, R)
        else:
            dz, dg, dbeta = dA, None, None
        fork.join()
        return None, dz, dg, dbeta, dW, db


def hanc_layer(x, weight, bias, k: int, *, consumer_bn=None):
    x = as_pending(x)
    pro = _finalize(x)
    B, H, W, C = x.z.shape
    w2 = weight.reshape(weight.shape[0], -1)
    N = w2.shape[0]
    assert w2.shape[1] == (2 * k - 1) * C
    if k >= 2 and (H % (2 if k == 2 else 4) or W % (2 if k == 2 else 4)):
        raise ValueError("HANCLayer: spatial size must be divisible by the pooling factor")
    want = _want_stats(consumer_bn)
    cfg = _HancCfg(pro, k, B, H, W, C, N, want, _bias_slot(bias, consumer_bn))
    pg, pb = _bn_params(x)
    Z, stats = _HancLayerFn.apply(cfg, x.z, pg, pb, w2, bias)
    return Pending(Z, consumer_bn, ACT_LRELU, stats if want else None,
                   stats.shape[0] if want else 0, bslot=cfg.bslot)


# --------------------------------------------------------------------------
# y = act(bn(z)) (+ res), materialised, optional statistics of y
# --------------------------------------------------------------------------
@dataclass
class _BAACfg:
    pro: _Pro
    has_res: bool
    want_stats: bool
    res_slot: object = None  # GradSlot collecting res's gradient


class _BnActAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg: _BAACfg, z, pro_g, pro_b, res):
        C = z.shape[-1]
        P = z.numel() // C
        y = torch.empty_like(z)
        stats = _stats((kern.stream_rows(P, C), 2, C), z) if cfg.want_stats else None
        pro = cfg.pro
        kern.affine_act(z, pro.st[2] if pro.active else None, pro.st[3] if pro.active else None,
                        pro.act if pro.active else ACT_NONE, res if cfg.has_res else None, y, P,
                        C, stats)
        ctx.cfg = cfg
        ctx.save_for_backward(z, pro_g)
        if stats is None:
            stats = _f32((0,), z)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _ds):
        if dy is None:  # output unused: every input gradient is zero
            sl = ctx.cfg.res_slot
            return (None,) * 4 + (sl.done() if sl is not None else None,)
        cfg = ctx.cfg
        z, pro_g = ctx.saved_tensors
        dy = dy.contiguous()
        dz, dg, db = _pro_bwd(cfg.pro, z, pro_g, dy)
        dres = dy if cfg.has_res else None
        if cfg.res_slot is not None:  # dy joins the shared buffer as a read-only addend
            cfg.res_slot.give(dy)
            dres = cfg.res_slot.done()
        return None, dz, dg, db, dres


def bn_act_add(x, res=None, *, consumer_bn=None, act_after=ACT_LRELU, want_stats=None,
               res_slot=None):
    """Materialise act(bn(x)) (+res); returns Pending(y, consumer_bn) with y's stats.
    res_slot: GradSlot collecting res's gradient (shared with res's other consumers)."""
    x = as_pending(x)
    pro = _finalize(x)
    if want_stats is None:
        want_stats = _want_stats(consumer_bn)
    cfg = _BAACfg(pro, res is not None, want_stats,
                  _slot_reg(res_slot) if res is not None else None)
    pg, pb = _bn_params(x)
    y, stats = _BnActAddFn.apply(cfg, x.z, pg, pb, res)
    C = y.shape[-1]
    return Pending(y, consumer_bn, act_after, stats if want_stats else None,
                   kern.stream_rows(y.numel() // C, C) if want_stats else 0)


# --------------------------------------------------------------------------
# ChannelSELayer (ACC_UNet/ACC_UNet.py:37-49) fused with its preceding BN(+act)
# --------------------------------------------------------------------------
@dataclass
class _SECfg:
    pro: _Pro
    bn: object  # the SE's own BatchNorm2d (running stats updated in forward)
    training: bool
    B: int
    HW: int
    C: int
    Cr: int
    want_stats: bool = False
    has_res: bool = False  # out = SE(x) + res (the fused residual add)
    res_slot: object = None  # GradSlot collecting res's gradient


class _SEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg: _SECfg, z, pro_g, pro_b, w1, b1, w2, b2, g, b, res):
        B, HW, C, Cr = cfg.B, cfg.HW, cfg.C, cfg.Cr
        pro = cfg.pro
        out = torch.empty_like(z)
        ostats = _stats((kern.se_stats_rows(B, HW, C), 2, C), z) if cfg.want_stats else None
        save = _f32((kern.se_save_elems(B, C, Cr),), z)
        bn = cfg.bn
        mom = bn.momentum if bn.momentum is not None else 0.1
        tr = cfg.training
        with _prof.region(f"se_fwd B{B} HW{HW} C{C}", kernel="se_reduce+se_mid_sample+se_apply",
                          shape=f"{B}x{HW}x{C}", bytes_alg=2.0 * z.element_size() * B * HW * C):
            kern.se_fwd(z, pro.st[2] if pro.active else None,
                        pro.st[3] if pro.active else None, pro.act, B, HW, C, Cr, w1, b1, w2,
                        b2, g, b, bn.running_mean if bn.track_running_stats else None,
                        bn.running_var if bn.track_running_stats else None,
                        bn.num_batches_tracked if (tr and bn.track_running_stats) else None,
                        mom, bn.eps, tr, out, save, ostats, res=res if cfg.has_res else None)
        ctx.cfg = cfg
        ctx.save_for_backward(z, pro_g, w1, w2, g, save)
        if ostats is None:
            ostats = _f32((0,), z)
        ctx.mark_non_differentiable(ostats)
        ctx.set_materialize_grads(False)
        return out, ostats

    @staticmethod
    def backward(ctx, dout, _dst):
        if dout is None:  # output unused: every input gradient is zero
            sl = ctx.cfg.res_slot
            return (None,) * 10 + (sl.done() if sl is not None else None,)
        cfg = ctx.cfg
        z, pro_g, w1, w2, g, save = ctx.saved_tensors
        dout = dout.contiguous()
        # the fused residual add: res's gradient is dout itself
        dres = dout if cfg.has_res else None
        if cfg.res_slot is not None:  # dout joins the shared buffer as a read-only addend
            cfg.res_slot.give(dout)
            dres = cfg.res_slot.done()
        B, HW, C, Cr = cfg.B, cfg.HW, cfg.C, cfg.Cr
        pro = cfg.pro
        dw1 = torch.empty_like(w1)
        db1 = _f32((Cr,), z)
        dw2 = torch.empty_like(w2)
        db2 = _f32((C,), z)
        dg = _f32((C,), z)
        dbeta = _f32((C,), z)
        if pro.active:
            # the preceding BatchNorm(+act)'s backward rides on the SE's two passes
            dz = torch.empty_like(z)
            dpg = _f32((C,), z)
            dpb = _f32((C,), z)
            dsum = _f32((C,), z) if pro.bslot is not None else None
            kern.se_bwd_pro(z, dout, pro.st, pro.act, pro_g, pro.training, B, HW, C, Cr, w1,
                            w2, g, cfg.training, save, dz, dpg, dpb, dw1, db1, dw2, db2, dg,
                            dbeta, dsum)
            if dsum is not None:
                pro.bslot.t = dsum
            return None, dz, dpg, dpb, dw1, db1, dw2, db2, dg, dbeta, dres
        da = torch.empty_like(z)
        kern.se_bwd(z, dout, None, None, pro.act, B, HW, C, Cr, w1, w2, g, cfg.training, save,
                    da, dw1, db1, dw2, db2, dg, dbeta)
        return None, da, None, None, dw1, db1, dw2, db2, dg, dbeta, dres


def se(x, mod, *, consumer_bn=None, res=None, res_slot=None):
    """ChannelSELayer `mod` (fc1, fc2, bn) applied to x (Pending or tensor), plus `res`
    when given: the residual add that follows the SE in ResPath and in the MLFC merge
    (ACC_UNet.py:326, :489-520), fused into the SE's apply pass, so the SE output is
    never written. res_slot: GradSlot collecting res's gradient.

    Returns the materialised output tensor, or (when consumer_bn is given) a
    Pending(out, consumer_bn) carrying the output's statistics."""
    x = as_pending(x)
    pro = _finalize(x)
    B, H, W, C = x.z.shape
    Cr = mod.fc1.weight.shape[0]
    bn = mod.bn
    tr = bn.training or not bn.track_running_stats
    want = _want_stats(consumer_bn)
    if res is not None:
        res = res.contiguous()
    cfg = _SECfg(pro, bn, tr, B, H * W, C, Cr, want, res is not None,
                 _slot_reg(res_slot) if res is not None else None)
    pg, pb = _bn_params(x)
    out, ostats = _SEFn.apply(cfg, x.z, pg, pb, mod.fc1.weight, mod.fc1.bias, mod.fc2.weight,
                              mod.fc2.bias, bn.weight, bn.bias, res)
    if consumer_bn is None:
        return out
    return Pending(out, consumer_bn, ACT_LRELU, ostats if want else None,
                   kern.se_stats_rows(B, H * W, C) if want else 0)


# --------------------------------------------------------------------------
# dense 3x3 conv, padding 1 (ResPath.convs, ACC_UNet/ACC_UNet.py:317-318,326)
# --------------------------------------------------------------------------
@dataclass
class _C3Cfg:
    B: int
    H: int
    W: int
    Cin: int
    Cout: int
    want_stats: bool
    bslot: object = None
    slot: object = None  # GradSlot collecting x's gradient


class _Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg: _C3Cfg, x, weight, bias):
        B, H, W, Ci, Co = cfg.B, cfg.H, cfg.W, cfg.Cin, cfg.Cout
        P = B * H * W
        Wr = _prepared(weight, "c3")
        if Wr is None:
            Wr = _f32((Co, 9 * Ci), x)  # [co][tap][ci]
            kern.permute4(weight, Wr, (Co, 3, 3, Ci), (9 * Ci, 3, 1, 9))
        Z = _act((B, H, W, Co), x)
        stats = _stats((kern.gemm_stats_rows(P, Co, 9 * Ci), 2, Co), x) if cfg.want_stats else None
        kern.gemm(P, Co, 9 * Ci, a=[x], lda=[Ci], amode=AMODE_SHIFT3, b=Wr, ldb=9 * Ci, c=Z,
                  ldc=Co, bias=bias, H=H, W=W, cin=Ci, stats=stats)
        ctx.cfg = cfg
        ctx.save_for_backward(x, weight)
        if stats is None:
            stats = _f32((0,), x)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)
        return Z, stats

    @staticmethod
    def backward(ctx, dZ, _ds):
        if dZ is None:  # output unused: every input gradient is zero
            return None, ctx.cfg.slot.done() if ctx.cfg.slot is not None else None, None, None
        cfg = ctx.cfg
        x, weight = ctx.saved_tensors
        dZ = dZ.contiguous()
        B, H, W, Ci, Co = cfg.B, cfg.H, cfg.W, cfg.Cin, cfg.Cout
        P = B * H * W
        keep = []
        dx = None
        dWr = _f32((Co, 9 * Ci), x)
        dW = torch.empty_like(weight)
        fork = _WgradFork(dZ, 2.0 * Co * 9 * Ci * P)
        with fork:  # weight gradient on the side stream (overlaps the data gradient)
            keep.append(kern.gemm(Co, 9 * Ci, P, a=[dZ], lda=[Co], amode=AMODE_COL, b=x, ldb=Ci,
                                  bmode=BMODE_NN_SHIFT3, c=dWr, ldc=9 * Ci, H=H, W=W, cin=Ci,
                                  allow_split=True))
            _wgrad_permute(dWr, dW, (Co, Ci, 3, 3), (9 * Ci, 1, 3 * Ci, Ci))
        if ctx.needs_input_grad[1]:
            Wf = _prepared(weight, "c3f")
            if Wf is None:
                Wf = _f32((Ci, 9 * Co), x)  # [ci][tap'][co] = W[co][ci][8-tap']
                kern.permute4(weight, Wf, (Ci, 3, 3, Co), (9, 3, 1, 9 * Ci), flips=(0, 1, 1, 0))
            if cfg.slot is None:
                dx, adds = torch.empty_like(x), []
            else:  # shared gradient buffer: earlier contributions are epilogue addends
                dx, adds = cfg.slot.gemm_target(x.shape, x)
            keep.append(kern.gemm(P, Ci, 9 * Co, a=[dZ], lda=[Co], amode=AMODE_SHIFT3, b=Wf,
                                  ldb=9 * Co, c=dx, ldc=Ci, H=H, W=W, cin=Co,
                                  ups=[(t, Ci, 0, 0) for t in adds]))
        if cfg.slot is not None:
            dx = cfg.slot.done()
        db = _take_bias_grad(cfg.bslot)
        if db is None:
            db = _f32((Co,), x)
            keep.append(kern.colsum(dZ, P, Co, db))
        fork.join()
        return None, dx, dW, db


def conv3x3(x: torch.Tensor, weight, bias, *, consumer_bn=None, slot=None):
    """slot: GradSlot collecting x's gradient (shared with x's other consumers)."""
    B, H, W, Ci = x.shape
    Co = weight.shape[0]
    want = _want_stats(consumer_bn)
    cfg = _C3Cfg(B, H, W, Ci, Co, want, _bias_slot(bias, consumer_bn), _slot_reg(slot))
    Z, stats = _Conv3x3Fn.apply(cfg, x, weight, bias)
    return Pending(Z, consumer_bn, ACT_LRELU, stats if want else None,
                   stats.shape[0] if want else 0, bslot=cfg.bslot)


# --------------------------------------------------------------------------
# ConvTranspose2d(k=2, s=2) (ACC_UNet/ACC_UNet.py:578-590,637-648)
# --------------------------------------------------------------------------
class _ConvT2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        B, H, W, Ci = x.shape
        Co = weight.shape[1]
        P = B * H * W
        Wr = _prepared(weight, "ct")
        if Wr is None:
            Wr = _f32((Ci, 4 * Co), x)  # [ci][d][co], d = di*2+dj
            kern.permute4(weight, Wr, (Ci, 2, 2, Co), (4 * Co, 2, 1, 4))
        T = _act((B, H, W, 4 * Co), x)
        kern.gemm(P, 4 * Co, Ci, a=[x], lda=[Ci], b=Wr, ldb=4 * Co, bmode=BMODE_NN, c=T,
                  ldc=4 * Co)
        Y = _act((B, 2 * H, 2 * W, Co), x)
        kern.pixel_shuffle2(T, bias, Y, B, H, W, Co)
        ctx.save_for_backward(x, Wr)
        ctx.shape = (B, H, W, Ci, Co)
        return Y

    @staticmethod
    def backward(ctx, dY):
        x, Wr = ctx.saved_tensors
        B, H, W, Ci, Co = ctx.shape
        P = B * H * W
        dY = dY.contiguous()
        dT = _act((B, H, W, 4 * Co), dY)
        kern.pixel_shuffle2(dT, None, dY, B, H, W, Co, inverse=True)
        keep = []
        dx = None
        dWr = _f32((Ci, 4 * Co), x)
        dW = _f32((Ci, Co, 2, 2), x)
        fork = _WgradFork(dT, 2.0 * Ci * 4 * Co * P)
        with fork:  # weight gradient on the side stream (overlaps the data gradient)
            keep.append(kern.gemm(Ci, 4 * Co, P, a=[x], lda=[Ci], amode=AMODE_COL, b=dT,
                                  ldb=4 * Co, bmode=BMODE_NN, c=dWr, ldc=4 * Co, allow_split=True))
            _wgrad_permute(dWr, dW, (Ci, Co, 2, 2), (4 * Co, 1, 2 * Co, Co))
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            keep.append(kern.gemm(P, Ci, 4 * Co, a=[dT], lda=[4 * Co], b=Wr, ldb=4 * Co, c=dx,
                                  ldc=Ci))
        db = _f32((Co,), x)
        keep.append(kern.colsum(dY, B * 4 * H * W, Co, db))
        fork.join()
        return dx, dW, db


def conv_transpose2x2(x, weight, bias):
    return _ConvT2Fn.apply(x, weight, bias)


class _ConvTCatFn(torch.autograd.Function):
    """torch.cat([ConvTranspose2d(k=2, s=2)(x), skip], dim=1) (ACC_UNet.py:637-648): the
    ConvT GEMM, then ONE pass that pixel-shuffles (+bias) its output into the first Co
    channels of the concatenated tensor and copies skip into the rest (accunet_convt_cat);
    the up-sampled tensor is never materialised on its own. Backward: one pass splits
    the incoming gradient into dT (un-shuffled) and dskip, then the ConvT GEMMs; the bias
    gradient is the column sums of dT ([P*4][Co])."""

    @staticmethod
    def forward(ctx, x, weight, bias, skip):
        B, H, W, Ci = x.shape
        Co = weight.shape[1]
        Cs = skip.shape[-1]
        P = B * H * W
        Wr = _prepared(weight, "ct")
        if Wr is None:
            Wr = _f32((Ci, 4 * Co), x)  # [ci][d][co], d = di*2+dj
            kern.permute4(weight, Wr, (Ci, 2, 2, Co), (4 * Co, 2, 1, 4))
        T = _act((B, H, W, 4 * Co), x)
        kern.gemm(P, 4 * Co, Ci, a=[x], lda=[Ci], b=Wr, ldb=4 * Co, bmode=BMODE_NN, c=T,
                  ldc=4 * Co)
        Y = _act((B, 2 * H, 2 * W, Co + Cs), x)
        kern.convt_cat(T, bias, skip.contiguous(), Y, B, H, W, Co, Cs)
        ctx.save_for_backward(x, Wr)
        ctx.shape = (B, H, W, Ci, Co, Cs)
        return Y

    @staticmethod
    def backward(ctx, dY):
        x, Wr = ctx.saved_tensors
        B, H, W, Ci, Co, Cs = ctx.shape
        P = B * H * W
        dY = dY.contiguous()
        dT = _act((B, H, W, 4 * Co), dY)
        dskip = _act((B, 2 * H, 2 * W, Cs), dY) if ctx.needs_input_grad[3] else None
        kern.convt_cat(dT, None, dskip, dY, B, H, W, Co, Cs, inverse=True)
        keep = []
        dx = None
        dWr = _f32((Ci, 4 * Co), x)
        dW = _f32((Ci, Co, 2, 2), x)
        fork = _WgradFork(dT, 2.0 * Ci * 4 * Co * P)
        with fork:  # weight gradient on the side stream (overlaps the data gradient)
            keep.append(kern.gemm(Ci, 4 * Co, P, a=[x], lda=[Ci], amode=AMODE_COL, b=dT,
                                  ldb=4 * Co, bmode=BMODE_NN, c=dWr, ldc=4 * Co, allow_split=True))
            _wgrad_permute(dWr, dW, (Ci, Co, 2, 2), (4 * Co, 1, 2 * Co, Co))
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            keep.append(kern.gemm(P, Ci, 4 * Co, a=[dT], lda=[4 * Co], b=Wr, ldb=4 * Co, c=dx,
                                  ldc=Ci))
        db = _f32((Co,), x)
        keep.append(kern.colsum(dT, P * 4, Co, db))
        fork.join()
        return dx, dW, db, dskip


_CONVT_CAT = os.environ.get("ACCUNET_CONVT_CAT", "1") != "0"  # 0: ConvT, then cat (A/B)


def conv_transpose2x2_cat(x, weight, bias, skip):
    """torch.cat([ConvTranspose2d(x), skip], dim=1) in NHWC (the decoder's up + cat)."""
    if not _CONVT_CAT or weight.shape[1] % 4 or skip.shape[-1] % 4:
        return cat_channels(conv_transpose2x2(x, weight, bias), skip)
    return _ConvTCatFn.apply(x, weight, bias, skip)


# --------------------------------------------------------------------------
# MaxPool2d(2) / AvgPool2d(2)
# --------------------------------------------------------------------------
class _Pool2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mode, slot=None):
        B, H, W, C = x.shape
        if H % 2 or W % 2:
            raise ValueError("pool2: spatial size must be even")
        y = _act((B, H // 2, W // 2, C), x)
        kern.pool2_fwd(x, y, B, H, W, C, mode)
        ctx.mode = mode
        ctx.slot = slot
        if mode == kern.POOL_MAX:
            ctx.save_for_backward(x, y)
        else:
            ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        saved = ctx.saved_tensors
        x = saved[0]
        y = saved[1] if ctx.mode == kern.POOL_MAX else x
        B, H, W, C = x.shape
        if ctx.slot is None:
            dx = torch.empty_like(x)
            kern.pool2_bwd(x, y, dy.contiguous(), dx, B, H, W, C, ctx.mode)
            return dx, None, None
        if dy is None:
            return ctx.slot.done(), None, None
        dx, acc = ctx.slot.acc_target(x.shape, x)
        kern.pool2_bwd(x, y, dy.contiguous(), dx, B, H, W, C, ctx.mode, accumulate=acc)
        ctx.slot.flush()
        return ctx.slot.done(), None, None


def pool2(x, mode=kern.POOL_MAX, slot=None):
    """slot: GradSlot collecting x's gradient (shared with x's other consumers)."""
    return _Pool2Fn.apply(x, mode, _slot_reg(slot))


# --------------------------------------------------------------------------
# channel concat (decoder torch.cat([up, skip], dim=1))
# --------------------------------------------------------------------------
class _CatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        B, H, W, Ca = a.shape
        Cb = b.shape[-1]
        P = B * H * W
        y = _act((B, H, W, Ca + Cb), a)
        kern.slice_copy(a, Ca, 0, y, Ca + Cb, 0, P, Ca)
        kern.slice_copy(b, Cb, 0, y, Ca + Cb, Ca, P, Cb)
        ctx.dims = (P, Ca, Cb)
        return y

    @staticmethod
    def backward(ctx, dy):
        P, Ca, Cb = ctx.dims
        dy = dy.contiguous()
        da = db = None
        if ctx.needs_input_grad[0]:
            da = _act(dy.shape[:-1] + (Ca,), dy)
            kern.slice_copy(dy, Ca + Cb, 0, da, Ca, 0, P, Ca)
        if ctx.needs_input_grad[1]:
            db = _act(dy.shape[:-1] + (Cb,), dy)
            kern.slice_copy(dy, Ca + Cb, Ca, db, Cb, 0, P, Cb)
        return da, db


def cat_channels(a, b):
    return _CatFn.apply(a, b)


# --------------------------------------------------------------------------
# head: 1x1 conv to one channel (+ Sigmoid) (ACC_UNet/ACC_UNet.py:594-599,653-659)
# --------------------------------------------------------------------------
class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, sigm):
        B, H, W, C = x.shape
        y = _f32((B, H, W, 1), x)  # the model output stays fp32 (it feeds the loss)
        kern.head_fwd(x, w, b, sigm, y, B * H * W, C)
        ctx.sigm = sigm
        ctx.save_for_backward(x, w, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        B, H, W, C = x.shape
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        db = _f32((1,), x)
        ws = kern.head_bwd(x, w, y, dy.contiguous(), ctx.sigm, dx, dw, db, B * H * W, C)
        del ws
        return dx, dw, db, None


def head(x, weight, bias, sigmoid: bool):
    C = x.shape[-1]
    return _HeadFn.apply(x, weight.reshape(C), bias, bool(sigmoid))


# --------------------------------------------------------------------------
# ACC_UNet_W learnable merge y = m*W + x*(1-W) (ACC_UNet/ACC_UNet_w.py:497-522)
# --------------------------------------------------------------------------
class _WMergeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, w, want_stats):
        C = a.shape[-1]
        P = a.numel() // C
        y = torch.empty_like(a)
        stats = _stats((kern.stream_rows(P, C), 2, C), a) if want_stats else None
        kern.wmerge_fwd(a, b, w, y, P, C, stats)
        ctx.save_for_backward(a, b, w)
        if stats is None:
            stats = _f32((0,), a)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _ds):
        if dy is None:  # output unused: every input gradient is zero
            return (None,) * 4
        a, b, w = ctx.saved_tensors
        dy = dy.contiguous()
        da = torch.empty_like(a)
        db = torch.empty_like(b)
        kern.wmerge_bwd(dy, w, da, db, a.numel())
        dw = _f32((1,), a)
        ws = kern.dotdiff(dy, a, b, a.numel(), dw)
        del ws
        return da, db, dw, None


def wmerge(m, x, w, *, consumer_bn=None):
    want = _want_stats(consumer_bn)
    y, stats = _WMergeFn.apply(m, x, w, want)
    C = y.shape[-1]
    return Pending(y, consumer_bn, ACT_LRELU, stats if want else None,
                   kern.stream_rows(y.numel() // C, C) if want else 0)


# --------------------------------------------------------------------------
# weight column relayout (MLFC merge: channel 2c = x_c, 2c+1 = x, ACC_UNet.py:492)
# --------------------------------------------------------------------------
class _GroupRelayoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w2, J, order):
        N, K = w2.shape
        C = K // J
        ctx.meta = (N, C, J, list(order))
        pre = _prepared(w2, "grp") if (J, tuple(order)) == (2, (0, 1)) else None
        if pre is not None:  # made by the step's WeightPrep launch (a view: the buffer stays plain)
            return pre.view(N, K)
        out = _f32((N, K), w2)
        kern.group_relayout(w2, out, N, C, J, order)
        return out

    @staticmethod
    def backward(ctx, g):
        N, C, J, order = ctx.meta
        out = _f32((N, J * C), g)
        _wgrad_group_inverse(g.contiguous(), out, N, C, J, order)
        return out, None, None


def group_relayout(w2, J, order):
    return _GroupRelayoutFn.apply(w2, J, tuple(order))


# --------------------------------------------------------------------------
# NCHW <-> NHWC at the module boundary
# --------------------------------------------------------------------------
class _ToNHWCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        B, C, H, W = x.shape
        y = torch.empty((B, H, W, C), dtype=dtype, device=x.device)
        kern.permute4(x, y, (B, H, W, C), (C * H * W, W, 1, H * W))
        return y

    @staticmethod
    def backward(ctx, dy):
        B, H, W, C = dy.shape
        dx = _f32((B, C, H, W), dy)
        kern.permute4(dy.contiguous(), dx, (B, C, H, W), (H * W * C, 1, W * C, C))
        return dx, None


def to_nhwc(x, dtype=torch.float32):
    """NCHW input -> NHWC activations stored as `dtype` (fp32 or bf16)."""
    x = x.contiguous()
    if x.dtype != torch.float32:
        x = x.float()
    return _ToNHWCFn.apply(x, dtype)


class _ToNCHWFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y):
        B, H, W, C = y.shape
        x = _f32((B, C, H, W), y)  # module outputs are fp32 NCHW
        kern.permute4(y, x, (B, C, H, W), (H * W * C, 1, W * C, C))
        ctx.act_dtype = y.dtype
        return x

    @staticmethod
    def backward(ctx, dx):
        B, C, H, W = dx.shape
        dy = torch.empty((B, H, W, C), dtype=ctx.act_dtype, device=dx.device)
        kern.permute4(dx.contiguous(), dy, (B, H, W, C), (C * H * W, W, 1, H * W))
        return dy


def nhwc_to_nchw(y):
    B, H, W, C = y.shape
    if C == 1 and y.dtype == torch.float32:
        return y.view(B, 1, H, W)
    return _ToNCHWFn.apply(y.contiguous())


# --------------------------------------------------------------------------
# WeightedDiceBCE(0.5, 0.5) (Experiments/utils.py:140-171)
# --------------------------------------------------------------------------
class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, t, dice_w, bce_w):
        B = x.shape[0]
        N = x.numel() // B
        res = torch.zeros(8 + 2 * B, dtype=torch.float32, device=x.device)
        ws = kern.loss_fwd(x, t, B, N, dice_w, bce_w, res)
        del ws
        ctx.save_for_backward(x, t, res)
        ctx.w = (dice_w, bce_w)
        return res[0].clone(), res[1].clone(), res[2].clone()

    @staticmethod
    def backward(ctx, gl, _gd, _gb):
        x, t, res = ctx.saved_tensors
        B = x.shape[0]
        N = x.numel() // B
        dx = torch.empty_like(x)
        g = gl.reshape(1).contiguous().float() if gl is not None else None
        kern.loss_bwd(x, t, B, N, ctx.w[0], ctx.w[1], res, g, dx)
        return dx, None, None, None


def weighted_dice_bce(logits, truth, dice_weight=1.0, bce_weight=1.0):
    x = logits.contiguous().float()
    t = truth.contiguous().float().reshape(x.shape)
    loss, _, _ = _LossFn.apply(x, t, float(dice_weight), float(bce_weight))
    return loss


def weighted_dice_terms(logits, truth):
    """WeightedDiceLoss value (Experiments/utils.py:115-138) from the same kernel."""
    x = logits.contiguous().float()
    t = truth.contiguous().float().reshape(x.shape)
    B = x.shape[0]
    res = torch.zeros(8 + 2 * B, dtype=torch.float32, device=x.device)
    kern.loss_fwd(x, t, B, x.numel() // B, 1.0, 1.0, res)
    return res[1]
