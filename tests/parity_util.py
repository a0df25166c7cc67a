"""Shared helpers for the GPU parity tests: run the HIP model and the CPU oracle
on identical deterministic weights / inputs and compare outputs, loss, gradients
and BatchNorm running statistics."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import accunet_oracle as O  # noqa: E402

BUFFER_LEAVES = ("running_mean", "running_var", "num_batches_tracked")
BN_FED_BIAS = (".conv1.bias", ".conv2.bias", ".hnc.cnv.bias", ".conv3.bias", ".norm.bias")


def structurally_zero(name):
    if name.startswith("rspth") and ".convs." in name and name.endswith(".bias"):
        return True
    return name.endswith(BN_FED_BIAS)


def oracle_run(variant, sd, x, mask, dtype=torch.float64, training=True, n_classes=1):
    sdo = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
    params = {}
    for k, v in sdo.items():
        if not k.endswith(BUFFER_LEAVES):
            v.requires_grad_(True)
            params[k] = v
    out = O.forward(sdo, x.to(dtype), variant, training=training, n_classes=n_classes)
    loss = None
    if mask is not None:
        loss = O.dice_bce_loss(out, mask.to(dtype))
        loss.backward()
    grads = {k: (p.grad if p.grad is not None else torch.zeros_like(p)) for k, p in params.items()}
    return out.detach(), loss, grads, sdo


def compare_grads(hip_grads: dict, ref_grads: dict, rtol=2e-3, floor_frac=2e-3):
    """Returns list of (name, err, scale, tol, ok)."""
    per = {k: g.abs().mean().item() for k, g in ref_grads.items()}
    live = [v for k, v in per.items() if v > 0 and not structurally_zero(k)]
    med = float(np.median(live)) if live else 0.0
    rows = []
    for k, gr in ref_grads.items():
        gh = hip_grads[k].detach().double().cpu()
        gr = gr.detach().double()
        err = (gh - gr).abs().max().item()
        scale = gr.abs().max().item()
        if structurally_zero(k) or per[k] < 1e-4 * med:
            tol = 0.3 * med + 1e-7
            ok = gh.abs().mean().item() < tol
        else:
            tol = rtol * scale + floor_frac * med
            ok = err <= tol
        rows.append((k, err, scale, tol, ok))
    return rows
