"""Dataset / input pipeline of the path: the counterpart of the reference's
ImageToImage2D (Experiments/Load_Dataset.py:387-487), the loader that feeds
train_model.py:313-330.

On-disk format (as the reference reads it): {dataset_path}/images/*.npy holding
(4, H, W) arrays (channel 0 is used, :456-460) and {dataset_path}/masks/*.npy
holding (H, W) masks under the same file name. Files are visited in sorted order.

Two ways to read it:
  ImageToImage2D   drop-in torch Dataset with the reference's __getitem__ output
                   ({'image': (1,S,S) float32 z-scored, 'label': (S,S) int64 0/1},
                   fname); host-side numpy/torch, for DataLoader users.
  DeviceBatches    the MI355X path: per batch, the raw channel-0 planes and raw
                   masks are stacked into pinned host buffers, copied to HBM once
                   each, and prepared on the GPU by two HIP launches
                   (accunet_image_prep: INTER_LINEAR resize if needed + per-image
                   z-score; accunet_mask_prep: INTER_NEAREST resize + binarise),
                   yielding ({'image': [B,1,S,S], 'label': [B,1,S,S] fp32}, names)
                   batches already resident on the device.

cv2 is not part of this image: resizing follows cv2's INTER_LINEAR / INTER_NEAREST
rules for float data (half-pixel centres, clamped; floor(dst * in / out)), which
torch's F.interpolate(bilinear, align_corners=False) / (nearest) also implement;
no reference fixture pins the resize (parity unpinned for that branch; the
tests check the HIP kernels against F.interpolate). Integer-typed raw planes are
interpolated as fp32 here, whereas cv2 interpolates in the native dtype and
rounds (parity unpinned). Non-square raw inputs are refused: the reference
resizes only when the height differs (Load_Dataset.py:467,481).
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import kern


def _list_npy(path: str) -> List[str]:
    return sorted(f for f in os.listdir(path) if f.endswith(".npy"))


def _load(path: str) -> np.ndarray:
    return np.load(path, allow_pickle=False)


class ImageToImage2D(torch.utils.data.Dataset):
    """Load_Dataset.py:387-487 (the active __getitem__, :453-487)."""

    def __init__(self, dataset_path: str, image_size: int = 256, channel_idx: int = 0):
        self.image_size = image_size
        self.channel_idx = channel_idx
        self.input_path = os.path.join(dataset_path, "images")
        self.output_path = os.path.join(dataset_path, "masks")
        self.images_list = _list_npy(self.input_path)

    def __len__(self):
        return len(self.images_list)

    def __getitem__(self, idx):
        fname = self.images_list[idx]
        S = self.image_size
        img = _load(os.path.join(self.input_path, fname))[self.channel_idx]
        img = torch.from_numpy(np.ascontiguousarray(img)).float()
        if img.shape[0] != S:
            img = F.interpolate(img[None, None], size=(S, S), mode="bilinear",
                                align_corners=False)[0, 0]
        img = img.unsqueeze(0)
        img = (img - img.mean()) / (img.std() + 1e-8)
        mask = _load(os.path.join(self.output_path, fname))
        m = torch.from_numpy(np.ascontiguousarray(mask))
        if m.shape[0] != S:
            m = F.interpolate(m[None, None].float(), size=(S, S), mode="nearest")[0, 0]
        m = (m > 0).long()
        return {"image": img, "label": m}, fname


_MASK_DT = {np.dtype(np.uint8): 0, np.dtype(np.bool_): 0, np.dtype(np.float32): 1,
            np.dtype(np.int64): 2}


class DeviceBatches:
    """Iterates a dataset directory in batches prepared on the GPU (see module doc).

    shuffle uses a torch.Generator seeded per epoch (the reference's DataLoader
    shuffles the training set, train_model.py:318-320)."""

    def __init__(self, dataset_path: str, batch_size: int, image_size: int = 256,
                 channel_idx: int = 0, shuffle: bool = False, seed: int = 0,
                 device: Optional[torch.device] = None):
        self.input_path = os.path.join(dataset_path, "images")
        self.output_path = os.path.join(dataset_path, "masks")
        self.names = _list_npy(self.input_path)
        self.batch_size = batch_size
        self.S = image_size
        self.channel_idx = channel_idx
        self.shuffle = shuffle
        self.seed = seed
        self.epoch = 0
        self.device = device or torch.device("cuda", torch.cuda.current_device())

    def __len__(self):
        return (len(self.names) + self.batch_size - 1) // self.batch_size

    def _batch(self, names):
        imgs = [_load(os.path.join(self.input_path, n))[self.channel_idx] for n in names]
        masks = [_load(os.path.join(self.output_path, n)) for n in names]
        hin, win = imgs[0].shape
        if any(i.shape != (hin, win) for i in imgs):
            raise ValueError("DeviceBatches: images of one batch must share their raw size")
        mh, mw = masks[0].shape
        # the reference resizes only when the HEIGHT differs from S (Load_Dataset.py:467,
        # :481), so a non-square raw plane with H == S would stay non-square there; the
        # device kernels write S x S, so such inputs are refused rather than resampled
        if hin != win or mh != mw:
            raise ValueError("DeviceBatches: raw images and masks must be square "
                             f"(got {hin}x{win} / {mh}x{mw}); Load_Dataset.py resizes on height only")
        mdt = masks[0].dtype
        if any(m.shape != (mh, mw) or m.dtype != mdt for m in masks):
            raise ValueError("DeviceBatches: masks of one batch must share size and dtype")
        if mdt not in _MASK_DT:
            masks = [m.astype(np.float32) for m in masks]
            mdt = np.dtype(np.float32)
        raw_i = torch.from_numpy(np.stack(imgs).astype(np.float32, copy=False)).pin_memory()
        raw_m = torch.from_numpy(np.stack(masks).view(np.uint8) if mdt == np.bool_
                                 else np.stack(masks)).pin_memory()
        B = len(names)
        di = raw_i.to(self.device, non_blocking=True)
        dm = raw_m.to(self.device, non_blocking=True)
        img = torch.empty(B, 1, self.S, self.S, dtype=torch.float32, device=self.device)
        lab = torch.empty(B, 1, self.S, self.S, dtype=torch.float32, device=self.device)
        kern.image_prep(di, B, hin, win, self.S, img)
        kern.mask_prep(dm, _MASK_DT[mdt], B, mh, mw, self.S, lab)
        return {"image": img, "label": lab}, list(names)

    def __iter__(self):
        order = list(range(len(self.names)))
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            order = torch.randperm(len(order), generator=g).tolist()
        self.epoch += 1
        for s in range(0, len(order), self.batch_size):
            yield self._batch([self.names[i] for i in order[s:s + self.batch_size]])
