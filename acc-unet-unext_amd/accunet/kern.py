"""Thin typed wrappers over the C ABI: torch tensors in, device pointers out.

Only plumbing lives here (pointer extraction, shape checks, workspace from the
PyTorch caching allocator, current HIP stream). All arithmetic is done by the
HIP kernels of libaccunet_hip.so.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import torch

from . import _lib
from ._lib import AccGemmDesc, call


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t: Optional[torch.Tensor]):
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


_DT = {torch.float32: _lib.ACC_F32, torch.bfloat16: _lib.ACC_BF16}


def _check(t: torch.Tensor, name: str, act: bool = False):
    """Device tensor of fp32 (or, for activation operands, act=True, fp32 / bf16)."""
    if not t.is_cuda:
        raise _lib.AccError(f"{name}: expected a device tensor (HIP), got {t.device}")
    if t.dtype != torch.float32 and not (act and t.dtype == torch.bfloat16):
        raise _lib.AccError(f"{name}: expected float32{' or bfloat16' if act else ''}, "
                            f"got {t.dtype}")


def _dt(t: torch.Tensor) -> int:
    """ACC_F32 / ACC_BF16 storage code of an activation tensor (include/accunet.h)."""
    try:
        return _DT[t.dtype]
    except KeyError:
        raise _lib.AccError(f"activation storage must be float32 or bfloat16, got {t.dtype}")


def _same_dt(ref: torch.Tensor, *ts):
    for t in ts:
        if t is not None and t.dtype != ref.dtype:
            raise _lib.AccError(f"mixed activation storage: {t.dtype} vs {ref.dtype}")
    return _dt(ref)


# marker ids accunet_graph_marker accepts (ACC_MAX_MARKERS in csrc/misc.hip)
MAX_GRAPH_MARKERS = 32


class GraphEvent:
    """A hipEvent_t for the graph-mode all-reduce gating (see include/accunet.h,
    accunet_graph_events_after_markers): `mark(id)` during capture leaves marker id
    in the stream; `attach(graph, events)` after capture adds an event-record node
    behind each marker; `wait(stream)` gates another stream on the event."""

    def __init__(self):
        h = ctypes.c_void_p()
        call("accunet_event_create", ctypes.byref(h))
        self.h = h

    @staticmethod
    def mark(marker_id: int, stream=None):
        s = (stream or torch.cuda.current_stream()).cuda_stream
        call("accunet_graph_marker", int(marker_id), ctypes.c_void_p(s))

    @staticmethod
    def attach(raw_graph: int, events) -> int:
        """add an event-record node behind each marker of the captured graph"""
        arr = (ctypes.c_void_p * len(events))(*[e.h.value for e in events])
        n = _lib.load().accunet_graph_events_after_markers(ctypes.c_void_p(raw_graph), arr,
                                                             len(events))
        if n < 0:
            raise _lib.AccError(f"accunet_graph_events_after_markers failed: {n}")
        return n

    def wait(self, stream):
        call("accunet_stream_wait_event", ctypes.c_void_p(stream.cuda_stream), self.h)

    def synchronize(self):
        call("accunet_event_synchronize", self.h)

    def __del__(self):
        try:
            if self.h:
                _lib.load().accunet_event_destroy(self.h)
        except Exception:
            pass


def workspace(n_elems: int, device, dtype=torch.float32) -> torch.Tensor:
    return torch.empty(max(int(n_elems), 1), dtype=dtype, device=device)


def stats_buffer(rows: int, C: int, device) -> torch.Tensor:
    return torch.empty(rows, 2, C, dtype=torch.float64, device=device)


def gemm(M: int, N: int, K: int, *, a: Sequence[torch.Tensor], lda: Sequence[int],
         kbeg: Optional[Sequence[int]] = None, amode: int = _lib.AMODE_ROW,
         b: torch.Tensor, ldb: int, bmode: int = _lib.BMODE_NT,
         c: torch.Tensor, ldc: int, bias: Optional[torch.Tensor] = None,
         pro_a: int = _lib.PRO_NONE, a_scale=None, a_shift=None,
         pro_b: int = _lib.PRO_NONE, b_scale=None, b_shift=None,
         H: int = 1, W: int = 1, cin: int = 0,
         ups: Sequence = (), stats: Optional[torch.Tensor] = None,
         allow_split: bool = False, a_offsets: Optional[Sequence[int]] = None,
         b_offset: int = 0, c_offset: int = 0, pyr: Optional[Sequence] = None,
         bnb: Optional[Sequence] = None):
    """C[M,N] = A(M,K) B(K,N) (+bias) (+ups) on the current stream.

    `ups` is a sequence of (tensor, ld, log2_factor, col_offset) nearest-upsample addends.
    Offsets are element offsets into the respective tensors (column slices).
    `pyr` = (dP2, dP4 or None, mk2, mk4 or None): HANCLayer pyramid backward fused into
    the epilogue (H, W = image size; see AccGemmDesc.pd2).
    `bnb` = (z, st, act): `stats` receives the BatchNorm-backward partials of the
    BatchNorm(+act) whose pre-BN input is z [M][ldc] (see AccGemmDesc.bz).
    """
    d = AccGemmDesc()
    d.M, d.N, d.K = int(M), int(N), int(K)
    d.amode, d.bmode, d.pro_a, d.pro_b = amode, bmode, pro_a, pro_b
    d.nsrc = len(a)
    offs = a_offsets or [0] * len(a)
    for i, (t, ld) in enumerate(zip(a, lda)):
        _check(t, "gemm.a", act=True)
        d.a[i] = t.data_ptr() + t.element_size() * int(offs[i])
        d.lda[i] = int(ld)
    d.adt = _same_dt(a[0], *a[1:])
    if kbeg is None:
        kbeg = [0, K]
    for i, v in enumerate(kbeg):
        d.kbeg[i] = int(v)
    d.a_scale = a_scale.data_ptr() if a_scale is not None else None
    d.a_shift = a_shift.data_ptr() if a_shift is not None else None
    _check(b, "gemm.b", act=True)
    d.b = b.data_ptr() + b.element_size() * int(b_offset)
    d.bdt = _dt(b)
    d.ldb = int(ldb)
    d.b_scale = b_scale.data_ptr() if b_scale is not None else None
    d.b_shift = b_shift.data_ptr() if b_shift is not None else None
    d.H, d.W, d.cin = int(H), int(W), int(cin)
    _check(c, "gemm.c", act=True)
    d.c = c.data_ptr() + c.element_size() * int(c_offset)
    d.cdt = _dt(c)
    d.ldc = int(ldc)
    d.bias = bias.data_ptr() if bias is not None else None
    d.nup = len(ups)
    for i, u in enumerate(ups):
        t, ld, lg = u[0], u[1], u[2]
        off = u[3] if len(u) > 3 else 0
        _same_dt(c, t)
        d.up[i] = t.data_ptr() + t.element_size() * int(off)
        d.upld[i] = int(ld)
        d.uplog[i] = int(lg)
    if stats is not None and stats.dtype != torch.float64:
        raise _lib.AccError("gemm.stats: fp64 partial-statistics buffer expected")
    d.stats = stats.data_ptr() if stats is not None else None
    d.allow_split = 1 if allow_split else 0
    if pyr is not None:
        pd2, pd4, mk2, mk4 = pyr
        _check(pd2, "gemm.pd2", act=True)
        _same_dt(c, pd2, pd4)
        if mk2.dtype != torch.uint8 or (mk4 is not None and mk4.dtype != torch.uint8):
            raise _lib.AccError("gemm.pyr: uint8 first-max codes expected")
        d.pd2 = pd2.data_ptr()
        d.pd4 = pd4.data_ptr() if pd4 is not None else None
        d.mk2 = mk2.data_ptr()
        d.mk4 = mk4.data_ptr() if mk4 is not None else None
    if bnb is not None:
        bz, bst, bact = bnb
        _check(bz, "gemm.bz", act=True)
        _same_dt(c, bz)
        if stats is None:
            raise _lib.AccError("gemm.bnb needs a stats buffer")
        d.bz = bz.data_ptr()
        d.bst = bst.data_ptr()
        d.bact = int(bact)
    ws = None
    ws_elems = 0
    if allow_split:
        # room for up to 1024 K-slabs (the driver targets ~1024 workgroups), capped at 256 MB
        ws_elems = min(1024, max(1, K // 64)) * M * N
        ws_elems = min(ws_elems, 1 << 26)
        ws = workspace(ws_elems, c.device)
    call("accunet_gemm", ctypes.byref(d), _p(ws), ws_elems, _stream())
    return ws  # keep alive until the stream consumes it (caching allocator is stream-ordered)


def gemm_stats_rows(M, N, K, amode=_lib.AMODE_ROW, bmode=_lib.BMODE_NT, cin=0) -> int:
    """partial-statistics rows accunet_gemm writes for an M x N x K GEMM."""
    return int(_lib.load().accunet_gemm_stats_rows(int(M), int(N), int(K), amode, bmode, int(cin)))


def stream_rows(P: int, C: int) -> int:
    return int(_lib.load().accunet_stream_rows(int(P), int(C)))


def partial_ws_elems(R: int, Wd: int) -> int:
    """mirror of accunet_partials_ws_elems (csrc/bn.hip)."""
    import math
    r1 = math.ceil(R / 32)
    return (r1 + math.ceil(r1 / 32) + 2) * Wd


def bn_finalize(part: Optional[torch.Tensor], R: int, C: int, count: float, gamma, beta,
                rmean, rvar, nbt, momentum: float, eps: float, training: bool,
                st: torch.Tensor):
    ws = workspace(partial_ws_elems(R, 2 * C), st.device, torch.float64) if training else None
    call("accunet_bn_finalize", _p(part), int(R), int(C), float(count), _p(gamma), _p(beta),
         _p(rmean), _p(rvar), _p(nbt), float(momentum), float(eps), 1 if training else 0,
         _p(st), _p(ws), _stream())
    return ws


def affine_act(x: torch.Tensor, sc, sh, act: int, res, y: torch.Tensor, P: int, C: int,
               stats: Optional[torch.Tensor] = None) -> int:
    rows = ctypes.c_int(0)
    call("accunet_affine_act_fwd", _p(x), _p(sc), _p(sh), int(act), _p(res), _p(y), int(P),
         int(C), _p(stats), ctypes.byref(rows), _same_dt(x, res, y), _stream())
    return rows.value


def bn_bwd(x, dy, st, gamma, act: int, training: bool, P: int, C: int, dx, accumulate: bool,
           dgamma, dbeta, dsum=None):
    """BatchNorm(+act) backward; dsum (optional [C]) receives sum_p dx."""
    ws_elems = int(_lib.load().accunet_bn_bwd_ws_elems(int(P), int(C)))
    ws = workspace(ws_elems, x.device)
    call("accunet_bn_bwd", _p(x), _p(dy), _p(st), _p(gamma), int(act), 1 if training else 0,
         int(P), int(C), _p(dx), 1 if accumulate else 0, _p(dgamma), _p(dbeta), _p(dsum),
         _p(ws), ws_elems, _same_dt(x, dy, dx), _stream())
    return ws


def bn_bwd_part(x, dy, st, gamma, act: int, training: bool, P: int, C: int, part, R: int, dx,
                dgamma, dbeta, dsum=None):
    """BatchNorm backward from producer-side partials part [R][2][C] (fp64); dsum
    (optional [C]) receives sum_p dx."""
    ws_elems = int(_lib.load().accunet_bn_bwd_part_ws_elems(int(P), int(R), int(C)))
    ws = workspace(ws_elems, x.device)
    call("accunet_bn_bwd_part", _p(x), _p(dy), _p(st), _p(gamma), int(act), 1 if training else 0,
         int(P), int(C), _p(part), int(R), _p(dx), _p(dgamma), _p(dbeta), _p(dsum), _p(ws),
         ws_elems, _same_dt(x, dy, dx), _stream())
    return ws


def colsum(x, P: int, C: int, out):
    nb = stream_rows(P, C)
    ws_elems = nb * 2 * C + partial_ws_elems(nb, 2 * C)
    ws = workspace(ws_elems, x.device, torch.float64)
    call("accunet_colsum", _p(x), int(P), int(C), _p(out), _p(ws), ws_elems, _dt(x), _stream())
    return ws


def reduce_stats(part, R: int, C: int, out2C):
    ws = workspace(partial_ws_elems(R, 2 * C), part.device, torch.float64)
    call("accunet_reduce_stats", _p(part), int(R), int(C), _p(out2C), _p(ws), _stream())
    return ws


def _lib_raw():
    return _lib.load()


def stream_ticket_bank(stream, bank: int) -> None:
    """Register the ticket bank of the statistics reductions enqueued on `stream`
    (a torch.cuda.Stream; accunet_stream_ticket_bank). Unregistered streams use bank 0."""
    call("accunet_stream_ticket_bank", ctypes.c_void_p(stream.cuda_stream), int(bank))


def dw3x3_rows(B, H, W, C, like: torch.Tensor, bnb: bool = False) -> int:
    """rows of the statistics partials accunet_dw3x3_fwd writes for this shape and like's
    storage dtype: the forward's (bnb False) or the BN-backward data gradient's"""
    return int(_lib_raw().accunet_dw3x3_rows(B, H, W, C, _dt(like), 1 if bnb else 0))


_DW_NAMES = {4: "dw3x3_os16_fwd_kernel", 3: "dw3x3_os_fwd_kernel", 2: "dw3x3_span_fwd_kernel", 1: "dw3x3_tile_fwd_kernel", 0: "dw3x3_fwd_kernel"}


def dw3x3_kernel_name(B, H, W, C, like=None) -> str:
    """the forward depthwise kernel accunet_dw3x3_fwd launches for this shape (and the
    storage dtype of `like`, fp32 if None)"""
    lib = _lib_raw()
    dt = _dt(like) if like is not None else _lib.ACC_F32
    return _DW_NAMES[int(lib.accunet_dw3x3_variant(B, H, W, C, dt))]


def copy_nt(src: torch.Tensor, dst: torch.Tensor):
    """non-temporal float4 copy of src's bytes into dst (the probes' streaming ceiling)"""
    n = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < n:
        raise _lib.AccError("copy_nt: destination smaller than the source")
    call("accunet_copy_nt", _p(src), _p(dst), int(n), _stream())


def dw3x3_fwd(x, wt, bias, sc, sh, act, flip, z, stats, B, H, W, C, bnb=None):
    """bnb = (bz, bst, bact): `stats` receives BatchNorm-backward partials (see
    accunet_dw3x3_fwd in include/accunet.h)."""
    bz, bst, bact = bnb if bnb is not None else (None, None, 0)
    call("accunet_dw3x3_fwd", _p(x), _p(wt), _p(bias), _p(sc), _p(sh), int(act), int(flip), _p(z),
         _p(stats), B, H, W, C, _p(bz), _p(bst), int(bact), _same_dt(x, z, bz), _stream())


def dw3x3_wgrad(x, dz, sc, sh, act, dw, db, B, H, W, C):
    n = int(_lib_raw().accunet_dw3x3_wgrad_ws(B, H, W, C, _same_dt(x, dz)))
    ws = workspace(n, x.device)
    call("accunet_dw3x3_wgrad", _p(x), _p(dz), _p(sc), _p(sh), int(act), _p(dw), _p(db), B, H, W,
         C, _p(ws), n, _same_dt(x, dz), _stream())
    return ws


def hanc_pyramid_fwd(x, sc, sh, act, B, H, W, C, k, p2, p4, mk2=None, mk4=None):
    call("accunet_hanc_pyramid_fwd", _p(x), _p(sc), _p(sh), int(act), B, H, W, C, k, _p(p2),
         _p(p4), None if mk2 is None else mk2.data_ptr(),
         None if mk4 is None else mk4.data_ptr(), _same_dt(x, p2, p4), _stream())


def hanc_pyramid_bwd(x, sc, sh, act, B, H, W, C, k, p2, p4, dp2, dp4, da):
    call("accunet_hanc_pyramid_bwd", _p(x), _p(sc), _p(sh), int(act), B, H, W, C, k, _p(p2),
         _p(p4), _p(dp2), _p(dp4), _p(da), _same_dt(x, p2, p4, dp2, dp4, da), _stream())


POOL_MAX, POOL_AVG = 0, 1


def pool2_fwd(x, y, B, H, W, C, mode):
    call("accunet_pool2_fwd", _p(x), _p(y), B, H, W, C, mode, _same_dt(x, y), _stream())


def pool2_bwd(x, y, dy, dx, B, H, W, C, mode, accumulate=False):
    call("accunet_pool2_bwd", _p(x), _p(y), _p(dy), _p(dx), B, H, W, C, mode,
         1 if accumulate else 0, _same_dt(x, y, dy, dx), _stream())


def upsample_bwd(inp, ld_in, in_off, out, ld_out, B, H, W, C, f, accumulate=False):
    call("accunet_upsample_bwd", _p(inp), int(ld_in), int(in_off), _p(out), int(ld_out), B, H, W,
         C, int(f), 1 if accumulate else 0, _same_dt(inp, out), _stream())


def upsample_bwd24(inp, ld_in, out2, ld_out2, out4, ld_out4, B, H, W, C):
    """2x2 and 4x4 block sums of inp in one pass (the bits of upsample_bwd f=2 and f=4)."""
    call("accunet_upsample_bwd24", _p(inp), int(ld_in), _p(out2), int(ld_out2), _p(out4),
         int(ld_out4), B, H, W, C, _same_dt(inp, out2, out4), _stream())


def slice_copy(src, ld_src, src_off, dst, ld_dst, dst_off, P, C, accumulate=False):
    call("accunet_slice_copy", _p(src), int(ld_src), int(src_off), _p(dst), int(ld_dst),
         int(dst_off), int(P), int(C), 1 if accumulate else 0, _same_dt(src, dst), _stream())


def pixel_shuffle2(t, bias, y, B, Hi, Wi, Cout, inverse=False):
    call("accunet_pixel_shuffle2", _p(t), _p(bias), _p(y), B, Hi, Wi, Cout, 1 if inverse else 0,
         _same_dt(t, y), _stream())


def convt_cat(t, bias, skip, y, B, Hi, Wi, Co, Cs, inverse=False):
    """ConvT pixel shuffle (+bias) and channel concat with skip in one pass
    (accunet_convt_cat); inverse: y is the gradient, t / skip receive theirs."""
    for name, x in (("t", t), ("y", y), ("skip", skip)):
        if x is not None and not x.is_contiguous():
            raise _lib.AccError(f"convt_cat: {name} must be contiguous")
    call("accunet_convt_cat", _p(t), _p(bias), _p(skip), _p(y), int(B), int(Hi), int(Wi), int(Co),
         int(Cs), 1 if inverse else 0, _same_dt(t, y, skip), _stream())


def permute4(inp, out, dims, strides, flips=None, accumulate=False):
    d = (ctypes.c_int * 4)(*[int(v) for v in dims])
    s = (ctypes.c_longlong * 4)(*[int(v) for v in strides])
    f = (ctypes.c_int * 4)(*[int(v) for v in (flips or (0, 0, 0, 0))])
    call("accunet_permute4", _p(inp), _p(out), d, s, f, 1 if accumulate else 0, _dt(inp),
         _dt(out), _stream())


def relayout_blocks(total: int) -> int:
    return int(_lib_raw().accunet_relayout_blocks(int(total)))


def relayout_batch(items_dev: torch.Tensor, n: int, nblocks: int):
    """one launch for n AccRelayout items already in device memory (WeightPrep)"""
    call("accunet_relayout_batch", _p(items_dev), int(n), int(nblocks), _stream())


def group_relayout(inp, out, N, C, J, order, inverse=False):
    o = (ctypes.c_int * 8)(*([int(v) for v in order] + [0] * (8 - len(order))))
    call("accunet_group_relayout", _p(inp), _p(out), int(N), int(C), int(J), o,
         1 if inverse else 0, _stream())


def se_save_elems(B, C, Cr) -> int:
    return int(_lib_raw().accunet_se_save_elems(B, C, Cr))


def se_ws_elems(B, HW, C, Cr) -> int:
    return int(_lib_raw().accunet_se_ws_elems(B, HW, C, Cr))


def se_stats_rows(B, HW, C) -> int:
    return int(_lib_raw().accunet_se_stats_rows(B, HW, C))


def se_fwd(z, sc, sh, act, B, HW, C, Cr, w1, b1, w2, b2, gamma, beta, rmean, rvar, nbt, momentum,
           eps, training, out, save, ostats=None, res=None):
    """res: out = SE(z) + res (the fused residual add, see accunet_se_fwd)."""
    n = se_ws_elems(B, HW, C, Cr)
    ws = workspace(n, z.device)
    if res is not None and (res.shape != z.shape or res.dtype != z.dtype or not res.is_contiguous()):
        raise ValueError("se_fwd: res must be a contiguous tensor shaped and typed like z")
    call("accunet_se_fwd", _p(z), _p(sc), _p(sh), int(act), B, HW, C, Cr, _p(w1), _p(b1), _p(w2),
         _p(b2), _p(gamma), _p(beta), _p(rmean), _p(rvar), _p(nbt), float(momentum), float(eps),
         1 if training else 0, _p(out), _p(res), _p(save), _p(ostats), _p(ws), n,
         _same_dt(z, out), _stream())
    return ws


def se_bwd(z, dout, sc, sh, act, B, HW, C, Cr, w1, w2, gamma, training, save, da, dw1, db1, dw2,
           db2, dgamma, dbeta):
    n = se_ws_elems(B, HW, C, Cr)
    ws = workspace(n, z.device)
    call("accunet_se_bwd", _p(z), _p(dout), _p(sc), _p(sh), int(act), B, HW, C, Cr, _p(w1),
         _p(w2), _p(gamma), 1 if training else 0, _p(save), _p(da), _p(dw1), _p(db1), _p(dw2),
         _p(db2), _p(dgamma), _p(dbeta), _p(ws), n, _same_dt(z, dout, da), _stream())
    return ws


def se_bwd_pro(z, dout, pst, act, pgamma, ptraining, B, HW, C, Cr, w1, w2, gamma, training, save,
               dz, dpgamma, dpbeta, dw1, db1, dw2, db2, dgamma, dbeta, dsum=None):
    """SE backward fused with the backward of its BatchNorm(+act) prologue (pst = [4][C]
    mean, rstd, scale, shift of that BatchNorm): writes dz and the prologue's dgamma/dbeta."""
    n = se_ws_elems(B, HW, C, Cr)
    ws = workspace(n, z.device)
    call("accunet_se_bwd_pro", _p(z), _p(dout), _p(pst), int(act), _p(pgamma),
         1 if ptraining else 0, B, HW, C, Cr, _p(w1), _p(w2), _p(gamma), 1 if training else 0,
         _p(save), _p(dz), _p(dpgamma), _p(dpbeta), _p(dsum), _p(dw1), _p(db1), _p(dw2), _p(db2),
         _p(dgamma), _p(dbeta), _p(ws), n, _same_dt(z, dout, dz), _stream())
    return ws


def head_fwd(x, w, b, sigm, y, P, C):
    call("accunet_head_fwd", _p(x), _p(w), _p(b), 1 if sigm else 0, _p(y), int(P), int(C),
         _dt(x), _stream())


def head_bwd(x, w, y, dy, sigm, dx, dw, db, P, C):
    n = int(_lib_raw().accunet_head_ws_elems(int(P), int(C)))
    ws = workspace(n, x.device)
    call("accunet_head_bwd", _p(x), _p(w), _p(y), _p(dy), 1 if sigm else 0, _p(dx), _p(dw),
         _p(db), int(P), int(C), _p(ws), n, _same_dt(x, dx), _stream())
    return ws


def loss_fwd(x, t, B, N, dice_w, bce_w, res):
    n = int(_lib_raw().accunet_loss_ws_elems(int(B)))
    ws = workspace(n, x.device)
    call("accunet_loss_fwd", _p(x), _p(t), int(B), int(N), float(dice_w), float(bce_w), _p(res),
         _p(ws), n, _stream())
    return ws


def loss_bwd(x, t, B, N, dice_w, bce_w, res, gout, dx):
    call("accunet_loss_bwd", _p(x), _p(t), int(B), int(N), float(dice_w), float(bce_w), _p(res),
         _p(gout), _p(dx), _stream())


def adam_chunk_elems() -> int:
    return int(_lib_raw().accunet_adam_chunk_elems())


def adam_step(table, chunk_t, chunk_s, nchunks, lr, b1, b2, eps, wd, step):
    call("accunet_adam_step", _p(table), _p(chunk_t), _p(chunk_s), int(nchunks), float(lr),
         float(b1), float(b2), float(eps), float(wd), int(step), _stream())


def dotdiff(g, a, b, n, out, accumulate=False):
    ws = workspace(1024, g.device)
    call("accunet_dotdiff", _p(g), _p(a), _p(b), int(n), _p(out), 1 if accumulate else 0, _p(ws),
         _same_dt(g, a, b), _stream())
    return ws


def wmerge_fwd(a, b, w, y, P, C, stats=None):
    call("accunet_wmerge_fwd", _p(a), _p(b), _p(w), _p(y), int(P), int(C), _p(stats),
         _same_dt(a, b, y), _stream())


def wmerge_bwd(g, w, da, db, n):
    call("accunet_wmerge_bwd", _p(g), _p(w), _p(da), _p(db), int(n), _same_dt(g, da, db),
         _stream())


def image_prep(raw, N, Hin, Win, S, out):
    """raw [N,Hin,Win] fp32 planes -> out [N,1,S,S]: INTER_LINEAR resize + z-score."""
    _check(raw, "image_prep raw")
    _check(out, "image_prep out")
    if raw.numel() != N * Hin * Win or out.numel() != N * S * S:
        raise _lib.AccError("image_prep: shape mismatch")
    call("accunet_image_prep", _p(raw), N, Hin, Win, S, _p(out), _stream())


def mask_prep(raw, dtype_code, N, Hin, Win, S, out):
    """raw [N,Hin,Win] masks (uint8/bool 0, float32 1, int64 2) -> out fp32 {0,1}
    [N,1,S,S] (INTER_NEAREST resize + binarise)."""
    if not raw.is_cuda:
        raise _lib.AccError("mask_prep: expected a device tensor")
    _check(out, "mask_prep out")
    if raw.numel() != N * Hin * Win or out.numel() != N * S * S:
        raise _lib.AccError("mask_prep: shape mismatch")
    call("accunet_mask_prep", _p(raw), int(dtype_code), N, Hin, Win, S, _p(out), _stream())


def dwconvk_out_hw(H, W, kh, kw, ph, pw):
    oh, ow = ctypes.c_int(0), ctypes.c_int(0)
    call("accunet_dwconvk_out_hw", H, W, kh, kw, ph, pw, ctypes.byref(oh), ctypes.byref(ow))
    return oh.value, ow.value


def dwconvk_fwd(x, w, bias, out, N, C, H, W, kh, kw, ph, pw, replicate):
    for t, n in ((x, "x"), (w, "weight"), (out, "out")):
        _check(t, f"dwconvk_fwd {n}")
    call("accunet_dwconvk_fwd", _p(x), _p(w), _p(bias), _p(out), N, C, H, W, kh, kw, ph, pw,
         int(replicate), _stream())


def dwconvk_dgrad(dy, w, dx, N, C, H, W, kh, kw, ph, pw, replicate):
    n = _lib.load().accunet_dwconvk_dgrad_ws(N, C, H, W, kh, kw, ph, pw, int(replicate))
    ws = workspace(n, dy.device)
    call("accunet_dwconvk_dgrad", _p(dy), _p(w), _p(dx), N, C, H, W, kh, kw, ph, pw,
         int(replicate), _p(ws), ctypes.c_size_t(ws.numel()), _stream())


def dwconvk_wgrad(x, dy, dw, db, N, C, H, W, kh, kw, ph, pw, replicate):
    n = _lib.load().accunet_dwconvk_wgrad_ws(N, C, H, W, kh, kw, ph, pw)
    ws = workspace(n, x.device)
    call("accunet_dwconvk_wgrad", _p(x), _p(dy), _p(dw), _p(db), N, C, H, W, kh, kw, ph, pw,
         int(replicate), _p(ws), ctypes.c_size_t(ws.numel()), _stream())


# ----------------------------------------------------------------- UNeXt kernels
def layernorm_fwd(x, g, b, y, mr, P, C, eps):
    _check(x, "layernorm x")
    call("accunet_layernorm_fwd", _p(x), _p(g), _p(b), _p(y), _p(mr), P, C, float(eps), _stream())


def layernorm_bwd(x, g, mr, dy, dx, dgb, P, C):
    """dgb: [2*C] buffer receiving dgamma | dbeta."""
    R = int(_lib.load().accunet_layernorm_rows(P))
    part = workspace(R * 2 * C, x.device)
    call("accunet_layernorm_bwd", _p(x), _p(g), _p(mr), _p(dy), _p(dx), _p(dgb),
         _p(_flat(dgb, C)), _p(part), P, C, _stream())
    return part


def _flat(t, off):
    f = t.view(-1)
    return f.narrow(0, off, f.numel() - off)


def gelu_fwd(x, y):
    call("accunet_gelu_fwd", _p(x), _p(y), x.numel(), _stream())


def gelu_bwd(x, dy, dx):
    call("accunet_gelu_bwd", _p(x), _p(dy), _p(dx), x.numel(), _stream())


def token_shift(x, y, B, H, W, C, axis, direction, shift_size=5):
    call("accunet_token_shift", _p(x), _p(y), B, H, W, C, axis, direction, shift_size, _stream())


def up2_relu_add_fwd(x, skip, out, mask, B, H, W, C):
    call("accunet_up2_relu_add_fwd", _p(x), _p(skip), _p(out), _p(mask), B, H, W, C, _stream())


def up2_relu_bwd(dout, mask, dx, B, H, W, C):
    call("accunet_up2_relu_bwd", _p(dout), _p(mask), _p(dx), B, H, W, C, _stream())


def relu(x, dy, y):
    call("accunet_relu", _p(x), _p(dy), _p(y), x.numel(), _stream())


def subsample2(src, dst, B, H, W, C, bwd):
    call("accunet_subsample2", _p(src), _p(dst), B, H, W, C, int(bwd), _stream())
