"""RandomGenerator / ValGenerator (Experiments/Load_Dataset.py:19-117) against the
SciPy / NumPy oracle (oracle/augment_oracle.py): the host parameter draws in the
reference's random-call order, the kernel's coordinate formulas (pinned against
scipy.ndimage.rotate / np.rot90 + np.flip on CPU), and the HIP kernel bit-exact on
the GPU."""
import os
import random
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "acc-unet-unext_amd"))
import augment_oracle as AO  # noqa: E402
from accunet import augment as A  # noqa: E402


def _seed(s):
    random.seed(s)
    np.random.seed(s)


def test_draws_follow_reference_call_order():
    _seed(3)
    mine = [A.draw_params() for _ in range(400)]
    _seed(3)
    ref = [AO.draw() for _ in range(400)]
    assert mine == ref
    modes = {m for m, *_ in mine}
    assert modes == {0, 1, 2}


@pytest.mark.parametrize("S", [5, 32, 64, 97])
def test_rotation_formula_matches_scipy(S):
    rng = np.random.default_rng(S)
    x = rng.integers(1, 256, (S, S), dtype=np.uint8)
    for angle in range(-20, 20):
        rot, off = A.rotation_affine(angle, S)
        np.testing.assert_array_equal(AO.rotate_affine_map(x, rot, off), AO.rotate(x, angle))


@pytest.mark.parametrize("S", [4, 7, 16])
def test_rot_flip_index_map_matches_numpy(S):
    x = np.arange(S * S, dtype=np.int64).reshape(S, S)
    for k in range(4):
        for axis in range(2):
            np.testing.assert_array_equal(AO.rot_flip_index_map(x, k, axis), AO.rot_flip(x, k, axis))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.uint8, torch.float32])
def test_augment_batch_bit_exact(dtype):
    rng = np.random.default_rng(11)
    B, S, C = 24, 64, 3
    imgs = rng.integers(0, 256, (B, S, S, C), dtype=np.uint8)
    prms, ref = [], []
    for b in range(B):
        if b < 8:
            mode, k, axis, angle = 1, b % 4, (b // 4) % 2, 0
        elif b < 20:
            mode, k, axis, angle = 2, 0, 0, [-20, -13, -7, -1, 0, 1, 5, 9, 13, 17, 19, -19][b - 8]
        else:
            mode, k, axis, angle = 0, 0, 0, 0
        prms.append(A.make_param(mode, k, axis, angle, S))
        ref.append(AO.geom(imgs[b], mode, k, axis, angle))
    x = torch.from_numpy(imgs).cuda()
    if dtype == torch.float32:
        x = x.float()
    out = A.augment_batch(x, prms).cpu().numpy()
    np.testing.assert_array_equal(out, np.stack(ref).astype(out.dtype))
    # single-channel planes ([B,1,S,S]) as DeviceBatches yields them
    y = torch.from_numpy(imgs[..., 0].astype(np.float32)).cuda()[:, None]
    outy = A.augment_batch(y, prms).cpu().numpy()[:, 0]
    np.testing.assert_array_equal(outy, np.stack([r[..., 0] for r in ref]).astype(np.float32))


@pytest.mark.gpu
def test_random_and_val_generators_match_oracle():
    rng = np.random.default_rng(5)
    out_size = (64, 64)
    for trial in range(12):
        S = 64 if trial % 3 else 48  # grayscale mismatch exercises the resize branch
        rgb = trial % 3 != 0
        img = rng.integers(0, 256, (S, S, 3) if rgb else (S, S), dtype=np.uint8)
        lab = (rng.random((S, S)) < 0.3).astype(np.uint8)
        sample = {"image": img, "label": lab}
        _seed(100 + trial)
        got = A.RandomGenerator(out_size)(dict(sample))
        _seed(100 + trial)
        ref = AO.random_generator(dict(sample), out_size)
        np.testing.assert_array_equal(got["image"].cpu().numpy(), ref["image"])
        np.testing.assert_array_equal(got["label"].cpu().numpy(), ref["label"])
        assert got["label"].dtype == torch.int64
        vg = A.ValGenerator(out_size)(dict(sample))
        vr = AO.val_generator(dict(sample), out_size)
        np.testing.assert_array_equal(vg["image"].cpu().numpy(), vr["image"])
        np.testing.assert_array_equal(vg["label"].cpu().numpy(), vr["label"])
