"""CPU oracle for the training augmentation (TEST INFRASTRUCTURE ONLY: imported by
tests/ alone, never by the product path).

Restates Experiments/Load_Dataset.py:19-117 with NumPy / SciPy (torchvision and PIL
are absent here; the reference only uses them to convert uint8 arrays to PIL
images and back, F.to_pil_image / F.to_tensor, which for uint8 HxW / HxWxC input
is the identity on the pixel values followed by a /255 float conversion):
  random_rot_flip  :19-26   k ~ randint(0,4), axis ~ randint(0,2) (np.random),
                            np.rot90(x, k) then np.flip(axis)
  random_rotate    :28-32   angle ~ randint(-20,20), ndimage.rotate(order=0,
                            reshape=False)
  RandomGenerator  :33-76   random.random() > 0.5 -> rot_flip, elif a second
                            random.random() < 0.5 -> rotate; zoom to output_size
                            (order 3 image / order 0 label) when the size differs;
                            image -> (C,H,W) float / 255, label -> int64
  ValGenerator     :78-108  zoom + conversion only
Parity is pinned by SciPy / NumPy themselves (the reference's own libraries), not by
a reference-held fixture: none exists for these transforms.
"""
import random

import numpy as np
from scipy import ndimage


def rot_flip(x, k, axis):
    return np.flip(np.rot90(x, k), axis=axis).copy()


def rotate(x, angle):
    return ndimage.rotate(x, angle, order=0, reshape=False)


def draw():
    """(mode, k, axis, angle) in the reference's call order"""
    if random.random() > 0.5:
        k = np.random.randint(0, 4)
        axis = np.random.randint(0, 2)
        return 1, int(k), int(axis), 0
    if random.random() < 0.5:
        return 2, 0, 0, int(np.random.randint(-20, 20))
    return 0, 0, 0, 0


def geom(x, mode, k, axis, angle):
    if mode == 1:
        return rot_flip(x, k, axis)
    if mode == 2:
        return rotate(x, angle)
    return x.copy()


def finish(img, lab, size0, output_size):
    x, y = size0
    if x != output_size[0] or y != output_size[1]:
        img = ndimage.zoom(img, (output_size[0] / x, output_size[1] / y), order=3)
        lab = ndimage.zoom(lab, (output_size[0] / x, output_size[1] / y), order=0)
    im = img.astype(np.float32) / np.float32(255.0)
    im = np.transpose(im, (2, 0, 1)) if im.ndim == 3 else im[None]
    return {"image": im, "label": lab.astype(np.int64)}


def random_generator(sample, output_size):
    img, lab = sample["image"], sample["label"]
    size0 = (img.shape[1], img.shape[0])
    mode, k, axis, angle = draw()
    return finish(geom(img, mode, k, axis, angle), geom(lab, mode, k, axis, angle), size0,
                  output_size)


def val_generator(sample, output_size):
    img, lab = sample["image"], sample["label"]
    return finish(img, lab, (img.shape[1], img.shape[0]), output_size)


def rotate_affine_map(x, rot, offset):
    """ndimage.rotate(order=0, reshape=False, mode='constant') restated as the
    kernel evaluates it: source = rot @ (r, c) + offset (unfused fp64, left to right),
    taken iff both coordinates are in [0, n-1], at floor(coord + 0.5)"""
    S = x.shape[0]
    r, c = np.meshgrid(np.arange(S, dtype=np.float64), np.arange(S, dtype=np.float64),
                       indexing="ij")
    y = rot[0, 0] * r + rot[0, 1] * c + offset[0]
    z = rot[1, 0] * r + rot[1, 1] * c + offset[1]
    ok = (y >= 0) & (y <= S - 1) & (z >= 0) & (z <= S - 1)
    yi = np.clip(np.floor(y + 0.5).astype(np.int64), 0, S - 1)
    zi = np.clip(np.floor(z + 0.5).astype(np.int64), 0, S - 1)
    out = np.zeros_like(x)
    out[ok] = x[yi[ok], zi[ok]]
    return out


def rot_flip_index_map(x, k, axis):
    """mode 1 restated as the kernel's inverse index map (undo the flip, then k
    quarter turns: rot90 maps out[i][j] = in[j][S-1-i])"""
    S = x.shape[0]
    out = np.empty_like(x)
    for r in range(S):
        for c in range(S):
            rr, cc = (S - 1 - r, c) if axis == 0 else (r, S - 1 - c)
            for _ in range(k & 3):
                rr, cc = cc, S - 1 - rr
            out[r, c] = x[rr, cc]
    return out
