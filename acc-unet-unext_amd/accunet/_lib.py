"""ctypes binding of libaccunet_hip.so (C ABI declared in include/accunet.h).

This is the Python side of the drop-in boundary: every compute call of the
ACC-UNet path goes through one of the `accunet_*` entry points below. There is
no fallback — if the shared library is missing or fails to load, importing the
ops raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_double, c_float, c_int, c_longlong, c_size_t, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libaccunet_hip.so")

# mirrors include/accunet.h enums
AMODE_ROW, AMODE_COL, AMODE_SHIFT3 = 0, 1, 2
BMODE_NT, BMODE_NN, BMODE_NN_SHIFT3 = 0, 1, 2
PRO_NONE, PRO_AFFINE, PRO_AFFINE_LRELU = 0, 1, 2
ACT_NONE, ACT_LRELU = 0, 1


class AccGemmDesc(Structure):
    _fields_ = [
        ("M", c_int), ("N", c_int), ("K", c_int),
        ("amode", c_int), ("bmode", c_int), ("pro_a", c_int), ("pro_b", c_int),
        ("nsrc", c_int),
        ("a", c_void_p * 4),
        ("lda", c_int * 4),
        ("kbeg", c_int * 5),
        ("a_scale", c_void_p), ("a_shift", c_void_p),
        ("b", c_void_p), ("ldb", c_int),
        ("b_scale", c_void_p), ("b_shift", c_void_p),
        ("H", c_int), ("W", c_int), ("cin", c_int),
        ("c", c_void_p), ("ldc", c_int),
        ("bias", c_void_p),
        ("nup", c_int),
        ("up", c_void_p * 3),
        ("upld", c_int * 3),
        ("uplog", c_int * 3),
        ("stats", c_void_p),
        ("allow_split", c_int),
    ]


P = c_void_p  # device pointer
I = c_int
L = c_longlong
F = c_float
D = c_double
S = c_size_t
IP = POINTER(c_int)

# name -> argtypes (restype is always int status)
_SIGS = {
    "accunet_gemm": [POINTER(AccGemmDesc), P, S, P],
    "accunet_gemm_stats_rows": [I, I, I, I, I],
    "accunet_stream_rows": [L, I],
    "accunet_bn_finalize": [P, I, I, D, P, P, P, P, P, F, F, I, P, P, P],
    "accunet_affine_act_fwd": [P, P, P, I, P, P, L, I, P, IP, P],
    "accunet_bn_bwd": [P, P, P, P, I, I, L, I, P, I, P, P, P, IP, P, S, P],
    "accunet_colsum": [P, L, I, P, P, S, P],
    "accunet_reduce_stats": [P, I, I, P, P, P],
}

_lib = None


class AccError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise AccError(
            f"libaccunet_hip.so not found at {LIB_PATH}; build it with "
            "`make -C acc-unet-unext_amd -j8` (or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = c_int
    _lib = lib
    return lib


def declared_symbols():
    return list(_SIGS)


_ERRS = {-1: "bad shape", -2: "bad argument / workspace too small", -3: "kernel launch failure"}


def check(status: int, what: str):
    if status != 0:
        raise AccError(f"{what} failed: {_ERRS.get(status, status)}")


def call(name: str, *args):
    lib = load()
    check(getattr(lib, name)(*args), name)
