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


def _check(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise _lib.AccError(f"{name}: expected a device tensor (HIP), got {t.device}")
    if t.dtype != torch.float32:
        raise _lib.AccError(f"{name}: expected float32, got {t.dtype}")


def workspace(n_elems: int, device) -> torch.Tensor:
    return torch.empty(max(int(n_elems), 1), dtype=torch.float32, device=device)


def stats_buffer(rows: int, C: int, device) -> torch.Tensor:
    return torch.empty(rows, 2, C, dtype=torch.float32, device=device)


def gemm(M: int, N: int, K: int, *, a: Sequence[torch.Tensor], lda: Sequence[int],
         kbeg: Optional[Sequence[int]] = None, amode: int = _lib.AMODE_ROW,
         b: torch.Tensor, ldb: int, bmode: int = _lib.BMODE_NT,
         c: torch.Tensor, ldc: int, bias: Optional[torch.Tensor] = None,
         pro_a: int = _lib.PRO_NONE, a_scale=None, a_shift=None,
         pro_b: int = _lib.PRO_NONE, b_scale=None, b_shift=None,
         H: int = 1, W: int = 1, cin: int = 0,
         ups: Sequence = (), stats: Optional[torch.Tensor] = None,
         allow_split: bool = False, a_offsets: Optional[Sequence[int]] = None,
         b_offset: int = 0, c_offset: int = 0):
    """C[M,N] = A(M,K) B(K,N) (+bias) (+ups) on the current stream.

    `ups` is a sequence of (tensor, ld, log2_factor, col_offset) nearest-upsample addends.
    Offsets are element offsets into the respective tensors (column slices).
    """
    d = AccGemmDesc()
    d.M, d.N, d.K = int(M), int(N), int(K)
    d.amode, d.bmode, d.pro_a, d.pro_b = amode, bmode, pro_a, pro_b
    d.nsrc = len(a)
    offs = a_offsets or [0] * len(a)
    for i, (t, ld) in enumerate(zip(a, lda)):
        _check(t, "gemm.a")
        d.a[i] = t.data_ptr() + 4 * int(offs[i])
        d.lda[i] = int(ld)
    if kbeg is None:
        kbeg = [0, K]
    for i, v in enumerate(kbeg):
        d.kbeg[i] = int(v)
    d.a_scale = a_scale.data_ptr() if a_scale is not None else None
    d.a_shift = a_shift.data_ptr() if a_shift is not None else None
    _check(b, "gemm.b")
    d.b = b.data_ptr() + 4 * int(b_offset)
    d.ldb = int(ldb)
    d.b_scale = b_scale.data_ptr() if b_scale is not None else None
    d.b_shift = b_shift.data_ptr() if b_shift is not None else None
    d.H, d.W, d.cin = int(H), int(W), int(cin)
    _check(c, "gemm.c")
    d.c = c.data_ptr() + 4 * int(c_offset)
    d.ldc = int(ldc)
    d.bias = bias.data_ptr() if bias is not None else None
    d.nup = len(ups)
    for i, u in enumerate(ups):
        t, ld, lg = u[0], u[1], u[2]
        off = u[3] if len(u) > 3 else 0
        d.up[i] = t.data_ptr() + 4 * int(off)
        d.upld[i] = int(ld)
        d.uplog[i] = int(lg)
    d.stats = stats.data_ptr() if stats is not None else None
    d.allow_split = 1 if allow_split else 0
    ws = None
    ws_elems = 0
    if allow_split:
        ws_elems = min(64, max(1, K // 64)) * M * N
        ws_elems = min(ws_elems, 1 << 26)
        ws = workspace(ws_elems, c.device)
    call("accunet_gemm", ctypes.byref(d), _p(ws), ws_elems, _stream())
    return ws  # keep alive until the stream consumes it (caching allocator is stream-ordered)


def gemm_stats_rows(M, N, amode=_lib.AMODE_ROW, bmode=_lib.BMODE_NT, cin=0) -> int:
    return int(_lib.load().accunet_gemm_stats_rows(int(M), int(N), amode, bmode, int(cin)))


def stream_rows(P: int, C: int) -> int:
    return int(_lib.load().accunet_stream_rows(int(P), int(C)))


def partial_ws_elems(R: int, Wd: int) -> int:
    import math
    r1 = math.ceil(R / 256)
    return (r1 + math.ceil(r1 / 256) + 2) * Wd


def bn_finalize(part: Optional[torch.Tensor], R: int, C: int, count: float, gamma, beta,
                rmean, rvar, nbt, momentum: float, eps: float, training: bool,
                st: torch.Tensor):
    ws = workspace(partial_ws_elems(R, 2 * C), st.device) if training else None
    call("accunet_bn_finalize", _p(part), int(R), int(C), float(count), _p(gamma), _p(beta),
         _p(rmean), _p(rvar), _p(nbt), float(momentum), float(eps), 1 if training else 0,
         _p(st), _p(ws), _stream())
    return ws


def affine_act(x: torch.Tensor, sc, sh, act: int, res, y: torch.Tensor, P: int, C: int,
               stats: Optional[torch.Tensor] = None) -> int:
    rows = ctypes.c_int(0)
    call("accunet_affine_act_fwd", _p(x), _p(sc), _p(sh), int(act), _p(res), _p(y), int(P),
         int(C), _p(stats), ctypes.byref(rows), _stream())
    return rows.value


def bn_bwd(x, dy, st, gamma, act: int, training: bool, P: int, C: int, dx, accumulate: bool,
           dgamma, dbeta, colsum=None):
    nb = stream_rows(P, C)
    ws_elems = nb * 2 * C + 3 * C + partial_ws_elems(nb, 2 * C)
    ws = workspace(ws_elems, x.device)
    rows = ctypes.c_int(0)
    call("accunet_bn_bwd", _p(x), _p(dy), _p(st), _p(gamma), int(act), 1 if training else 0,
         int(P), int(C), _p(dx), 1 if accumulate else 0, _p(dgamma), _p(dbeta), _p(colsum),
         ctypes.byref(rows), _p(ws), ws_elems, _stream())
    return ws


def colsum(x, P: int, C: int, out):
    nb = stream_rows(P, C)
    ws_elems = nb * 2 * C + partial_ws_elems(nb, 2 * C)
    ws = workspace(ws_elems, x.device)
    call("accunet_colsum", _p(x), int(P), int(C), _p(out), _p(ws), ws_elems, _stream())
    return ws


def reduce_stats(part, R: int, C: int, out2C):
    ws = workspace(partial_ws_elems(R, 2 * C), part.device)
    call("accunet_reduce_stats", _p(part), int(R), int(C), _p(out2C), _p(ws), _stream())
    return ws
