"""Input pipeline (accunet/data.py, csrc/data.hip) against the oracle restatement of
ImageToImage2D.__getitem__ (Experiments/Load_Dataset.py:453-487).

The image branch without resizing is pinned to plain torch arithmetic; the resize
branches restate cv2's INTER_LINEAR / INTER_NEAREST rules (cv2 is not installed,
no reference fixture covers them: parity unpinned there, cross-checked against
torch's F.interpolate, which implements the same rules)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import accunet_oracle as O  # noqa: E402

from accunet import data as D  # noqa: E402


def make_dataset(root, n, H, mask_dtype=np.uint8, seed=0):
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "images"))
    os.makedirs(os.path.join(root, "masks"))
    for i in range(n):
        img = (rng.standard_normal((4, H, H)) * (3 + i) + 10 * i).astype(np.float32)
        m = (rng.random((H, H)) < 0.3)
        m = (m * 255).astype(mask_dtype) if mask_dtype != np.bool_ else m
        np.save(os.path.join(root, "images", f"case{i:03d}.npy"), img)
        np.save(os.path.join(root, "masks", f"case{i:03d}.npy"), m)
    return root


def test_cv_resize_rules_match_torch_interpolate():
    rng = np.random.default_rng(1)
    for H, S in [(40, 64), (100, 64), (64, 64), (7, 16)]:
        img = rng.standard_normal((H, H)).astype(np.float32)
        ref = F.interpolate(torch.from_numpy(img)[None, None], size=(S, S), mode="bilinear",
                            align_corners=False)[0, 0].numpy()
        assert np.abs(O.cv_resize_linear(img, S) - ref).max() < 1e-5
        m = (rng.random((H, H)) < 0.5).astype(np.float32)
        refm = F.interpolate(torch.from_numpy(m)[None, None], size=(S, S), mode="nearest")[0, 0]
        assert np.array_equal(O.cv_resize_nearest(m, S), refm.numpy())


@pytest.mark.parametrize("H,S", [(32, 32), (48, 32), (20, 32)])
def test_dataset_matches_oracle(tmp_path, H, S):
    root = make_dataset(str(tmp_path / "ds"), 3, H)
    ds = D.ImageToImage2D(root, image_size=S)
    assert len(ds) == 3
    for i in range(3):
        (item, fname) = ds[i]
        assert fname == f"case{i:03d}.npy"
        img_raw = np.load(os.path.join(root, "images", fname))
        m_raw = np.load(os.path.join(root, "masks", fname))
        ti, tm = O.load_item(img_raw, m_raw, S)
        assert item["image"].shape == (1, S, S) and item["image"].dtype == torch.float32
        assert item["label"].shape == (S, S) and item["label"].dtype == torch.int64
        tol = 0 if H == S else 1e-5
        assert (item["image"] - ti).abs().max().item() <= tol
        assert torch.equal(item["label"], tm)


@pytest.mark.gpu
@pytest.mark.parametrize("H,S,mdt", [(32, 32, np.uint8), (48, 32, np.float32),
                                     (20, 32, np.bool_), (256, 256, np.int64)])
def test_device_batches_match_oracle(tmp_path, H, S, mdt):
    root = make_dataset(str(tmp_path / "ds"), 5, H, mask_dtype=mdt)
    db = D.DeviceBatches(root, batch_size=2, image_size=S, device=torch.device("cuda"))
    assert len(db) == 3
    seen = []
    for batch, names in db:
        assert batch["image"].is_cuda and batch["image"].shape[1:] == (1, S, S)
        for j, fname in enumerate(names):
            ti, tm = O.load_item(np.load(os.path.join(root, "images", fname)),
                                 np.load(os.path.join(root, "masks", fname)), S)
            got = batch["image"][j].cpu()
            assert (got - ti).abs().max().item() < 2e-5, fname
            assert torch.equal(batch["label"][j, 0].cpu(), tm.float()), fname
            seen.append(fname)
    assert seen == sorted(seen) and len(seen) == 5
    # shuffled epochs visit every file once, in a seed-dependent order
    db2 = D.DeviceBatches(root, batch_size=2, image_size=S, shuffle=True, seed=3,
                          device=torch.device("cuda"))
    order = [n for _, names in db2 for n in names]
    assert sorted(order) == seen


@pytest.mark.gpu
def test_device_batches_feed_the_trainer(tmp_path):
    """train_model.py end to end on .npy files: DeviceBatches -> Trainer(ACC_UNet with
    n_channels=1, as the single-channel loader implies) for two epochs."""
    from accunet.model import ACC_UNet
    from accunet.trainer import Trainer
    root = make_dataset(str(tmp_path / "ds"), 4, 48)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = ACC_UNet(1, 1, n_filts=8).to(dev)
    tr = Trainer(model, "ACC_UNet", str(tmp_path / "ck"), epochs=2)
    train = D.DeviceBatches(root, batch_size=2, image_size=32, shuffle=True, device=dev)
    val = D.DeviceBatches(root, batch_size=2, image_size=32, device=dev)
    tr.fit(train, val)
    assert [h["mode"] for h in tr.history] == ["Train", "Val", "Train", "Val"]
    assert all(np.isfinite(h["loss"]) and 0 <= h["dice"] <= 1 for h in tr.history)
