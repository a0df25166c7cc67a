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


def oracle_run_fp32_ensemble(variant, sd, x, mask, seeds=(1, 2, 3)):
    """The reference's fp32 arithmetic re-run on inputs and weights perturbed by one
    fp32 rounding (relative 2^-24 uniform noise, i.e. the error every fp32 program
    already makes when it stores them). Returns one dict per seed keyed like the
    tests' comparison dicts ("out", "grad:<name>", "buf:<name>"); the spread of these
    runs around the fp64 oracle measures each tensor's fp32 sensitivity (condition x
    eps), which a single fp32 run can under-state by several x on cancellation-
    dominated tensors (and which differs between CPUs' BLAS kernels)."""
    res = []
    for seed in seeds:
        g = torch.Generator().manual_seed(seed)

        def jit(t):
            if not t.is_floating_point():
                return t.clone()
            u = torch.rand(t.shape, generator=g, dtype=torch.float64) * 2 - 1
            return (t.double() * (1 + u * 2.0 ** -24)).to(t.dtype)
        sdp = {k: (v.clone() if k.endswith(BUFFER_LEAVES) else jit(v)) for k, v in sd.items()}
        out, _, grads, sdo = oracle_run(variant, sdp, jit(x), mask, dtype=torch.float32)
        d = {"out": out}
        for k, g in grads.items():
            d["grad:" + k] = g
        for k, v in sdo.items():
            if k.endswith(("running_mean", "running_var")):
                d["buf:" + k] = v
        res.append(d)
    return res


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


def compare_vs_reference_fp32(hip: dict, ref64: dict, ref32: dict, factor=4.0, rel_floor=1e-4,
                              abs_floor=None, ref32_extra=()):
    """Per-tensor check that the HIP fp32 result is as close to the fp64 oracle as the
    reference's own fp32 arithmetic is (oracle run in fp32 = same ATen ops as the
    reference): max|hip - ref64| <= factor * max|ref32 - ref64| + rel_floor * max|ref64|.
    ref32_extra: further fp32 runs (e.g. batch-permuted, oracle_run_fp32_ensemble);
    the reference error is then the max over all fp32 runs.
    Returns rows (name, err_hip, err_ref32, tol, ok)."""
    rows = []
    for k, r64 in ref64.items():
        r64 = r64.detach().double().cpu()
        h = hip[k].detach().double().cpu()
        r32 = ref32[k].detach().double().cpu()
        e_h = (h - r64).abs().max().item() if r64.numel() else 0.0
        e_r = (r32 - r64).abs().max().item() if r64.numel() else 0.0
        for extra in ref32_extra:
            if k in extra and r64.numel():
                e_r = max(e_r, (extra[k].detach().double().cpu() - r64).abs().max().item())
        scale = r64.abs().max().item() if r64.numel() else 0.0
        tol = factor * e_r + rel_floor * scale + 1e-9
        if abs_floor is not None:
            tol += abs_floor.get(k, 0.0) if isinstance(abs_floor, dict) else abs_floor
        rows.append((k, e_h, e_r, tol, e_h <= tol))
    return rows


def per_tensor_norm_rows(hip: dict, ref64: dict, ref32_runs, keys, factor=4.0, rel_floor=1e-6):
    """Per-tensor NORM check without absolute floors: ||hip - ref64|| <= factor *
    max_runs ||ref32 - ref64|| + rel_floor * ||ref64||, for every tensor in keys. A norm
    is far less noisy than a max, so this catches a small tensor whose gradient is
    wrong as a whole (which the max-based check's absolute floors could let pass).
    Returns rows (name, err_hip, err_ref32, tol, ok)."""
    rows = []
    for k in keys:
        r64 = ref64[k].detach().double().cpu()
        e_h = float((hip[k].detach().double().cpu() - r64).norm())
        e_r = max(float((run[k].detach().double().cpu() - r64).norm()) for run in ref32_runs
                  if k in run)
        tol = factor * e_r + rel_floor * float(r64.norm()) + 1e-12
        rows.append((k, e_h, e_r, tol, e_h <= tol))
    return rows


def global_rel_err(hip: dict, ref: dict, keys):
    num = sum(float((hip[k].detach().double().cpu() - ref[k].detach().double().cpu()).norm() ** 2)
              for k in keys)
    den = sum(float(ref[k].detach().double().cpu().norm() ** 2) for k in keys)
    return (num / max(den, 1e-300)) ** 0.5


def median_live_grad(ref_grads: dict) -> float:
    per = [g.abs().mean().item() for k, g in ref_grads.items()
           if g.numel() and not structurally_zero(k)]
    per = [v for v in per if v > 0]
    return float(np.median(per)) if per else 0.0


def grad_cosine(a: dict, b: dict, keys) -> float:
    """cosine of the angle between two whole gradient vectors (the direction test)"""
    num = sum(float((a[k].double().cpu() * b[k].double().cpu()).sum()) for k in keys)
    na = sum(float((a[k].double().cpu() ** 2).sum()) for k in keys)
    nb = sum(float((b[k].double().cpu() ** 2).sum()) for k in keys)
    return num / max((na * nb) ** 0.5, 1e-300)
