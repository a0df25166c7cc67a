"""Test-set evaluation: the counterpart of Experiments/test_model.py (:41-70 per
image, :210-250 the loop) for the models of this package.

Per image, in eval mode: pred = (output > 0.5) (the model's own output, a
probability for the sigmoid-headed presets), dice = 2 sum(l p) / (sum l + sum p +
1e-5) (show_image_with_dice, :30-38 — no smoothing in the numerator), IoU =
sklearn.jaccard_score(l, p) (0 when both masks are empty); the reported numbers are
the means over the test images (:246-250). The reference runs the loader at batch
size 1 and copies each prediction to the host; here any batch size works and the
per-image metrics are computed on the device, read once at the end.
"""
from __future__ import annotations

from typing import Iterable

import torch

from .trainer import load_checkpoint


@torch.no_grad()
def image_dice_iou(output: torch.Tensor, labels: torch.Tensor):
    """Per-image (dice, iou) device tensors for a batch: output [B,1,H,W], labels
    [B,H,W] or [B,1,H,W]."""
    B = output.shape[0]
    p = (output.reshape(B, -1) > 0.5).float()
    lab = labels.reshape(B, -1).float()
    inter = (lab * p).sum(1, dtype=torch.float64)
    dice = 2 * inter / (lab.sum(1, dtype=torch.float64) + p.sum(1, dtype=torch.float64) + 1e-5)
    lb, pb = lab > 0, p > 0
    i2 = (lb & pb).sum(1, dtype=torch.float64)
    u2 = (lb | pb).sum(1, dtype=torch.float64)
    iou = torch.where(u2 > 0, i2 / u2.clamp_min(1), torch.zeros_like(i2))
    return dice, iou


@torch.no_grad()
def evaluate(model: torch.nn.Module, loader: Iterable, device=None) -> dict:
    """test_model.py's loop: mean Dice / IoU over every image the loader yields."""
    device = device or next(model.parameters()).device
    model.eval()
    dices, ious, names_all = [], [], []
    for sampled_batch, names in loader:
        x = sampled_batch["image"].to(device, non_blocking=True)
        y = sampled_batch["label"].to(device, non_blocking=True)
        out = model(x)
        d, i = image_dice_iou(out, y)
        dices.append(d)
        ious.append(i)
        names_all += list(names)
    d = torch.cat(dices).cpu()
    i = torch.cat(ious).cpu()
    n = max(d.numel(), 1)
    return {"dice": float(d.sum()) / n, "iou": float(i.sum()) / n, "n": d.numel(),
            "per_image": {nm: (float(a), float(b)) for nm, a, b in zip(names_all, d, i)}}


def load_best(model: torch.nn.Module, path: str, map_location=None) -> torch.nn.Module:
    """test_model.py:183,226: load a best_model-*.pth.tar checkpoint's state_dict."""
    ck = load_checkpoint(path, map_location=map_location)
    model.load_state_dict(ck["state_dict"])
    return model
