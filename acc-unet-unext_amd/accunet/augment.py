"""Training augmentation: RandomGenerator / ValGenerator of
Experiments/Load_Dataset.py:19-117 (random_rot_flip :19-26, random_rotate :28-32).

Per sample the reference (a) converts image / label to PIL images, (b) with
probability 1/2 rotates by k*90 degrees (np.rot90, k ~ U{0..3}) and flips along
axis ~ U{0,1}; otherwise with probability 1/2 (a second draw) rotates by an
integer angle ~ U{-20..19} with scipy.ndimage.rotate(order=0, reshape=False)
(nearest, zero outside); (c) resizes with scipy.ndimage.zoom to output_size when
the size differs (image order 3, label order 0); (d) returns
{'image': to_tensor(image) (C,H,W) float in [0,1], 'label': int64 (H,W)}.
ValGenerator does (a), (c), (d).

Here the geometric step (b) runs on the GPU (csrc/augment.hip), for one sample or
for a whole device-resident batch with per-sample parameters (augment_batch): the
parameters are drawn from Python's `random` and NumPy's global generator in the
reference's call order, so seeding both reproduces the reference's choices; the
rotation matrix and offset are computed in fp64 as scipy computes them and the
kernel is bit-exact with scipy/numpy (tests/test_augment.py).
The resize (c) is host-side scipy.ndimage.zoom on the transformed sample, as in the
reference -- it is only reachable for grayscale planes (for an HxWx3 image the
reference's 2-factor zoom raises, and so does this one); no reference fixture
covers it beyond scipy itself. Inputs: uint8 images (H,W) or (H,W,C) and uint8
labels (H,W), square planes.
"""
from __future__ import annotations

import ctypes
import random
from typing import Optional, Sequence, Tuple

import numpy as np
import torch
from scipy import ndimage, special

from . import _lib

MODE_COPY, MODE_ROT_FLIP, MODE_ROTATE = 0, 1, 2


class AccAugParam(ctypes.Structure):
    _fields_ = [("r00", ctypes.c_double), ("r01", ctypes.c_double), ("r10", ctypes.c_double),
                ("r11", ctypes.c_double), ("o0", ctypes.c_double), ("o1", ctypes.c_double),
                ("mode", ctypes.c_int), ("k", ctypes.c_int), ("axis", ctypes.c_int),
                ("pad", ctypes.c_int)]


def draw_params():
    """One sample's transform, drawing from `random` and np.random in the order of
    RandomGenerator.__call__ (Load_Dataset.py:41-45): (mode, k, axis, angle)."""
    if random.random() > 0.5:
        k = int(np.random.randint(0, 4))
        axis = int(np.random.randint(0, 2))
        return MODE_ROT_FLIP, k, axis, 0
    if random.random() < 0.5:
        angle = int(np.random.randint(-20, 20))
        return MODE_ROTATE, 0, 0, angle
    return MODE_COPY, 0, 0, 0


def rotation_affine(angle: float, size: int) -> Tuple[np.ndarray, np.ndarray]:
    """scipy.ndimage.rotate's (reshape=False) source-coordinate map for a size x size
    plane: source = R @ (row, col) + offset (float64, scipy's own formulas)."""
    c, s = special.cosdg(angle), special.sindg(angle)
    rot = np.array([[c, s], [-s, c]])
    shape = np.array([size, size])
    offset = (shape - 1) / 2 - rot @ ((shape - 1) / 2)
    return rot, offset


def make_param(mode: int, k: int = 0, axis: int = 0, angle: float = 0.0, size: int = 1):
    p = AccAugParam()
    p.mode, p.k, p.axis = mode, k, axis
    if mode == MODE_ROTATE:
        rot, off = rotation_affine(angle, size)
        p.r00, p.r01, p.r10, p.r11 = (float(v) for v in rot.ravel())
        p.o0, p.o1 = float(off[0]), float(off[1])
    return p


def _param_tensor(params: Sequence[AccAugParam], device) -> torch.Tensor:
    raw = (AccAugParam * len(params))(*params)
    host = torch.frombuffer(bytearray(bytes(raw)), dtype=torch.uint8)
    return host.to(device)


def augment_batch(x: torch.Tensor, params: Sequence[AccAugParam]) -> torch.Tensor:
    """Apply per-sample transforms to a device batch [B, S, S] / [B, S, S, C] /
    [B, 1, S, S] (uint8 or float32); returns a new tensor of the same shape."""
    if not x.is_cuda:
        raise ValueError("augment_batch: the batch must be on the GPU")
    if x.dtype not in (torch.uint8, torch.float32):
        raise TypeError(f"augment_batch: uint8 or float32 batches, got {x.dtype}")
    x = x.contiguous()
    B = x.shape[0]
    if x.dim() == 4 and x.shape[1] == 1 and x.shape[2] == x.shape[3]:
        S, C = x.shape[2], 1
    elif x.dim() == 4:
        S, C = x.shape[1], x.shape[3]
        if x.shape[2] != S:
            raise ValueError(f"augment_batch: square planes only, got {tuple(x.shape)}")
    elif x.dim() == 3:
        S, C = x.shape[1], 1
        if x.shape[2] != S:
            raise ValueError(f"augment_batch: square planes only, got {tuple(x.shape)}")
    else:
        raise ValueError(f"augment_batch: bad shape {tuple(x.shape)}")
    if len(params) != B:
        raise ValueError(f"augment_batch: {len(params)} parameter blocks for a batch of {B}")
    out = torch.empty_like(x)
    prm = _param_tensor(params, x.device)
    dt = _lib.ACC_AUG_U8 if x.dtype == torch.uint8 else _lib.ACC_AUG_F32
    _lib.call("accunet_aug_geom", x.data_ptr(), out.data_ptr(), dt, B, S, C, prm.data_ptr(),
              torch.cuda.current_stream(x.device).cuda_stream)
    return out


def _as_u8(a, what):
    a = np.asarray(a)
    if a.dtype != np.uint8:
        raise TypeError(f"{what}: uint8 arrays (PIL-convertible), got {a.dtype}")
    if a.ndim not in (2, 3) or a.shape[0] != a.shape[1]:
        raise ValueError(f"{what}: square (H,W) or (H,W,C) planes, got {a.shape}")
    return a


def _geom(img: np.ndarray, lab: np.ndarray, prm: AccAugParam, device):
    ti = torch.from_numpy(np.ascontiguousarray(img)).to(device)
    tl = torch.from_numpy(np.ascontiguousarray(lab)).to(device)
    ti = augment_batch(ti[None], [prm])[0]
    tl = augment_batch(tl[None], [prm])[0]
    return ti, tl


_LUT = {}


def _u8_table(device):
    if device not in _LUT:
        _LUT[device] = (torch.arange(256, dtype=torch.float32) / 255.0).to(device)
    return _LUT[device]


def _finish(img_t: torch.Tensor, lab_t: torch.Tensor, size0: Tuple[int, int],
            output_size: Sequence[int]):
    """resize (host scipy zoom, Load_Dataset.py:47-54) + to_tensor / to_long_tensor"""
    x, y = size0  # PIL size = (width, height) of the input
    if x != output_size[0] or y != output_size[1]:
        img = ndimage.zoom(img_t.cpu().numpy(), (output_size[0] / x, output_size[1] / y), order=3)
        lab = ndimage.zoom(lab_t.cpu().numpy(), (output_size[0] / x, output_size[1] / y), order=0)
        img_t = torch.from_numpy(np.ascontiguousarray(img)).to(img_t.device)
        lab_t = torch.from_numpy(np.ascontiguousarray(lab)).to(lab_t.device)
    # uint8 -> float / 255 (F.to_tensor) by a table built with CPU (correctly
    # rounded) division: a device division differs from it in the last bit
    image = _u8_table(img_t.device)[img_t.long()]
    image = image.permute(2, 0, 1).contiguous() if image.dim() == 3 else image[None]
    return {"image": image, "label": lab_t.long()}


class RandomGenerator:
    """Load_Dataset.py:33-76 (drop-in callable on {'image', 'label'} samples)."""

    def __init__(self, output_size, device: Optional[torch.device] = None):
        self.output_size = output_size
        self.device = device or torch.device("cuda", torch.cuda.current_device())

    def __call__(self, sample):
        img = _as_u8(sample["image"], "RandomGenerator image")
        lab = _as_u8(sample["label"], "RandomGenerator label")
        size0 = (img.shape[1], img.shape[0])
        mode, k, axis, angle = draw_params()
        ti, tl = _geom(img, lab, make_param(mode, k, axis, angle, img.shape[0]), self.device)
        return _finish(ti, tl, size0, self.output_size)


class ValGenerator:
    """Load_Dataset.py:78-108: resize only."""

    def __init__(self, output_size, device: Optional[torch.device] = None):
        self.output_size = output_size
        self.device = device or torch.device("cuda", torch.cuda.current_device())

    def __call__(self, sample):
        img = _as_u8(sample["image"], "ValGenerator image")
        lab = _as_u8(sample["label"], "ValGenerator label")
        size0 = (img.shape[1], img.shape[0])
        ti = torch.from_numpy(np.ascontiguousarray(img)).to(self.device)
        tl = torch.from_numpy(np.ascontiguousarray(lab)).to(self.device)
        return _finish(ti, tl, size0, self.output_size)
