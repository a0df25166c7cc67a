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
# ACCUNET_LIB_OVERRIDE: A/B experiments against another build of the same library
# (tools/*_ab.sh); unset, the in-tree build is the only one ever loaded
_DEFAULT_LIB = os.path.join(_HERE, "libaccunet_hip.so")
LIB_PATH = os.environ.get("ACCUNET_LIB_OVERRIDE") or _DEFAULT_LIB

# mirrors include/accunet.h enums
AMODE_ROW, AMODE_COL, AMODE_SHIFT3 = 0, 1, 2
BMODE_NT, BMODE_NN, BMODE_NN_SHIFT3 = 0, 1, 2
PRO_NONE, PRO_AFFINE, PRO_AFFINE_LRELU = 0, 1, 2
ACT_NONE, ACT_LRELU = 0, 1
ACC_F32, ACC_BF16 = 0, 1
ACC_AUG_F32, ACC_AUG_U8 = 0, 1  # accunet_aug_geom element types


class AccRelayout(Structure):
    _fields_ = [
        ("inp", c_void_p), ("out", c_void_p), ("total", c_longlong), ("kind", c_int),
        ("blk0", c_int), ("d", c_int * 4), ("s", c_longlong * 4), ("flip", c_int * 4),
        ("N", c_int), ("C", c_int), ("J", c_int), ("order", c_int * 8), ("scale", c_float),
    ]


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
        ("stats", c_void_p),  # double*
        ("allow_split", c_int),
        ("pd2", c_void_p), ("pd4", c_void_p),  # fused pyramid backward (float*)
        ("mk2", c_void_p), ("mk4", c_void_p),  # first-max codes (uint8*)
        ("bz", c_void_p), ("bst", c_void_p), ("bact", c_int),  # BN-backward epilogue stats
        ("adt", c_int), ("bdt", c_int), ("cdt", c_int),  # storage: ACC_F32 / ACC_BF16
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
    "accunet_gemm_stats_rows": [I, I, I, I, I, I],
    "accunet_stream_rows": [L, I],
    "accunet_stream_ticket_bank": [P, I],
    "accunet_stream_ticket_unregister": [P],
    "accunet_abi_hash": [],
    "accunet_conv3x3_halo_launches": [I],
    "accunet_copy_nt": [P, P, L, P],
    "accunet_relayout_blocks": [L],
    "accunet_relayout_batch": [P, I, I, P],
    "accunet_bn_finalize": [P, I, I, D, P, P, P, P, P, F, F, I, P, P, P],
    "accunet_affine_act_fwd": [P, P, P, I, P, P, L, I, P, IP, I, P],
    "accunet_bn_bwd_ws_elems": [L, I],
    "accunet_bn_bwd": [P, P, P, P, I, I, L, I, P, I, P, P, P, P, S, I, P],
    "accunet_colsum": [P, L, I, P, P, S, I, P],
    "accunet_reduce_stats": [P, I, I, P, P, P],
    "accunet_dw3x3_rows": [I, I, I, I, I, I],
    "accunet_dw3x3_variant": [I, I, I, I, I],
    "accunet_dw3x3_fwd": [P, P, P, P, P, I, I, P, P, I, I, I, I, P, P, I, I, P],
    "accunet_bn_bwd_part_ws_elems": [L, I, I],
    "accunet_bn_bwd_part": [P, P, P, P, I, I, L, I, P, I, P, P, P, P, P, S, I, P],
    "accunet_dw3x3_wgrad_ws": [I, I, I, I, I],
    "accunet_dw3x3_wgrad": [P, P, P, P, I, P, P, I, I, I, I, P, S, I, P],
    "accunet_hanc_pyramid_fwd": [P, P, P, I, I, I, I, I, I, P, P, P, P, I, P],
    "accunet_hanc_pyramid_bwd": [P, P, P, I, I, I, I, I, I, P, P, P, P, P, I, P],
    "accunet_pool2_fwd": [P, P, I, I, I, I, I, I, P],
    "accunet_pool2_bwd": [P, P, P, P, I, I, I, I, I, I, I, P],
    "accunet_upsample_bwd": [P, I, I, P, I, I, I, I, I, I, I, I, P],
    "accunet_upsample_bwd24": [P, I, P, I, P, I, I, I, I, I, I, P],
    "accunet_slice_copy": [P, I, I, P, I, I, L, I, I, I, P],
    "accunet_pixel_shuffle2": [P, P, P, I, I, I, I, I, I, P],
    "accunet_convt_cat": [P, P, P, P, I, I, I, I, I, I, I, P],
    "accunet_permute4": [P, P, IP, POINTER(c_longlong), IP, I, I, I, P],
    "accunet_group_relayout": [P, P, I, I, I, IP, I, P],
    "accunet_se_save_elems": [I, I, I],
    "accunet_se_ws_elems": [I, I, I, I],
    "accunet_se_fwd": [P, P, P, I, I, I, I, I, P, P, P, P, P, P, P, P, P, F, F, I, P, P, P, P, P, S, I,
                       P],
    "accunet_se_stats_rows": [I, I, I],
    "accunet_se_bwd": [P, P, P, P, I, I, I, I, I, P, P, P, I, P, P, P, P, P, P, P, P, P, S, I, P],
    "accunet_se_bwd_pro": [P, P, P, I, P, I, I, I, I, I, P, P, P, I, P, P, P, P, P, P, P, P, P, P,
                           P, P, S, I, P],
    "accunet_head_fwd": [P, P, P, I, P, L, I, I, P],
    "accunet_head_ws_elems": [L, I],
    "accunet_head_bwd": [P, P, P, P, I, P, P, P, L, I, P, S, I, P],
    "accunet_loss_ws_elems": [I],
    "accunet_loss_fwd": [P, P, I, L, F, F, P, P, S, P],
    "accunet_loss_bwd": [P, P, I, L, F, F, P, P, P, P],
    "accunet_adam_chunk_elems": [],
    "accunet_adam_step": [P, P, P, I, F, F, F, F, F, I, P],
    "accunet_dotdiff": [P, P, P, L, P, I, P, I, P],
    "accunet_wmerge_fwd": [P, P, P, P, L, I, P, I, P],
    "accunet_wmerge_bwd": [P, P, P, P, L, I, P],
    "accunet_graph_marker": [I, P],
    "accunet_graph_events_after_markers": [P, POINTER(c_void_p), I],
    "accunet_event_create": [POINTER(c_void_p)],
    "accunet_event_destroy": [P],
    "accunet_stream_wait_event": [P, P],
    "accunet_event_synchronize": [P],
    "accunet_event_create_timed": [POINTER(c_void_p)],
    "accunet_graph_time_markers": [P, I, I, P, P, POINTER(c_void_p)],
    "accunet_graph_exec_event_set": [P, P, P],
    "accunet_event_elapsed_ms": [P, P, POINTER(c_float)],
    "accunet_image_prep": [P, I, I, I, I, P, P],
    "accunet_mask_prep": [P, I, I, I, I, I, P, P],
    "accunet_aug_geom": [P, P, I, I, I, I, P, P],
    "accunet_dwconvk_out_hw": [I, I, I, I, I, I, IP, IP],
    "accunet_layernorm_rows": [L],
    "accunet_layernorm_fwd": [P, P, P, P, P, L, I, F, P],
    "accunet_layernorm_bwd": [P, P, P, P, P, P, P, P, L, I, P],
    "accunet_gelu_fwd": [P, P, L, P],
    "accunet_gelu_bwd": [P, P, P, L, P],
    "accunet_token_shift": [P, P, I, I, I, I, I, I, I, P],
    "accunet_up2_relu_add_fwd": [P, P, P, P, I, I, I, I, P],
    "accunet_up2_relu_bwd": [P, P, P, I, I, I, I, P],
    "accunet_relu": [P, P, P, L, P],
    "accunet_subsample2": [P, P, I, I, I, I, I, P],
    "accunet_dwconvk_fwd": [P, P, P, P, I, I, I, I, I, I, I, I, I, P],
    "accunet_dwconvk_dgrad_ws": [I, I, I, I, I, I, I, I, I],
    "accunet_dwconvk_dgrad": [P, P, P, I, I, I, I, I, I, I, I, I, P, S, P],
    "accunet_dwconvk_wgrad_ws": [I, I, I, I, I, I, I, I],
    "accunet_dwconvk_wgrad": [P, P, P, P, I, I, I, I, I, I, I, I, I, P, S, P],
}
# entry points returning a size/count rather than a status
_SIZE_FNS = {"accunet_bn_bwd_ws_elems", "accunet_bn_bwd_part_ws_elems", "accunet_dw3x3_wgrad_ws", "accunet_se_save_elems", "accunet_se_ws_elems",
             "accunet_head_ws_elems", "accunet_loss_ws_elems", "accunet_dwconvk_wgrad_ws",
             "accunet_dwconvk_dgrad_ws"}

_LL_FNS = {"accunet_abi_hash", "accunet_conv3x3_halo_launches"}
HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "accunet.h")

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
    check_abi(lib)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = (c_size_t if name in _SIZE_FNS else c_longlong if name in _LL_FNS
                      else c_int)
    _lib = lib
    return lib


def header_abi_hash(path: str = HEADER) -> int:
    """The ABI identity the Makefile bakes into the library: the first 15 hex digits
    of include/accunet.h's sha256 (csrc/abi.hip)."""
    import hashlib
    with open(path, "rb") as fh:
        return int(hashlib.sha256(fh.read()).hexdigest()[:15], 16)


def check_abi(lib) -> None:
    """Refuse a library built from another header (an ACCUNET_LIB_OVERRIDE A/B build of
    older sources, or a stale in-tree build): its entry points would be called with
    this binding's argument lists, shifted wherever a signature changed."""
    if not hasattr(lib, "accunet_abi_hash"):
        raise AccError(f"{LIB_PATH} predates the ABI hash (accunet_abi_hash): rebuild it")
    lib.accunet_abi_hash.argtypes = []
    lib.accunet_abi_hash.restype = c_longlong
    got = int(lib.accunet_abi_hash())
    if os.path.exists(HEADER):
        want = header_abi_hash()
        if got != want:
            raise AccError(f"{LIB_PATH} was built from another include/accunet.h (ABI hash "
                           f"{got:#x}, header {want:#x}): rebuild it with "
                           "`make -C acc-unet-unext_amd`")
    elif LIB_PATH != _DEFAULT_LIB:
        raise AccError("ACCUNET_LIB_OVERRIDE needs include/accunet.h to check the ABI")


def declared_symbols():
    return list(_SIGS)


_ERRS = {-1: "bad shape", -2: "bad argument / workspace too small", -3: "kernel launch failure"}


def check(status: int, what: str):
    if status != 0:
        raise AccError(f"{what} failed: {_ERRS.get(status, status)}")


_DEBUG = os.environ.get("ACCUNET_DEBUG", "0") not in ("", "0")


def call(name: str, *args):
    lib = load()
    if _DEBUG:  # serialise + trace every entry point (debug builds of a run only)
        import sys
        import torch
        sys.stderr.write(f"[accunet] {name}\n")
        sys.stderr.flush()
    check(getattr(lib, name)(*args), name)
    if _DEBUG:
        torch.cuda.synchronize()
