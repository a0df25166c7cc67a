"""Generate the golden fixtures that pin the CPU oracle to the reference.

Run in the build container only (needs /root/reference):
    python tests/golden/make_golden.py               # every fixture
    python tests/golden/make_golden.py --fullwidth   # only the n_filts=32 ones (6)
    python tests/golden/make_golden.py --unext       # only the UNeXt ones (7)
It imports the reference modules from /root/reference (read-only), fills them
with the oracle's deterministic, version-independent parameters
(oracle/accunet_oracle.py: det_state_dict), runs them on deterministic inputs
and writes small .npz / .json fixtures next to this script. Only the fixtures
(data) are committed; the reference never leaves this container.
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import accunet_oracle as O  # noqa: E402


def load_module(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def ref_models():
    canon = load_module("ref_acc_unet", os.path.join(REF, "ACC_UNet/ACC_UNet.py"))
    script = load_module("ref_acc_unet_script", os.path.join(REF, "Experiments/nets/ACC_UNet.py"))
    lite = load_module("ref_acc_unet_lite", os.path.join(REF, "ACC_UNet/ACC_UNet_lite.py"))
    wmod = load_module("ref_acc_unet_w", os.path.join(REF, "ACC_UNet/ACC_UNet_w.py"))
    return {
        "canonical": canon.ACC_UNet,
        "script": script.ACC_UNet,
        "lite": lite.ACC_UNet_Lite,
        "w": wmod.ACC_UNet_W,
    }


def ref_utils():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))  # imported, never called (utils.py:9)
    return load_module("ref_utils", os.path.join(REF, "Experiments/utils.py"))


def ref_unext(U):
    """Experiments/nets/UNext.py with import shims for the packages this image lacks.
    Its forward path is the reference's own code plus torch; what the shims stand for:
      torchvision (transforms, utils.save_image): imported at :4,8-9, never called;
      timm.models.layers (:17): to_2tuple (:169-170) restated as timm defines it (an int
        -> (x, x)); trunc_normal_ (:58,131,184, weight init only, overwritten by
        load_state_dict) = torch.nn.init.trunc_normal_, the same algorithm; DropPath is
        only built for drop_path > 0 (:123; UNext's default drop_path_rate is 0), so the
        shim raises if it is ever constructed;
      `from utils import *` (:13): Experiments/utils.py itself (cv2 shim as above)."""
    import torch.nn as nn
    sys.modules["utils"] = U
    tv = types.ModuleType("torchvision")
    tv.transforms = types.ModuleType("torchvision.transforms")
    tvu = types.ModuleType("torchvision.utils")
    tvu.save_image = None
    tv.utils = tvu
    timm = types.ModuleType("timm")
    tmod = types.ModuleType("timm.models")
    layers = types.ModuleType("timm.models.layers")

    class DropPath(nn.Module):
        def __init__(self, *a, **k):
            raise RuntimeError("DropPath is not on the path at drop_path_rate 0")

    layers.DropPath = DropPath
    layers.to_2tuple = lambda x: tuple(x) if isinstance(x, (tuple, list)) else (x, x)
    layers.trunc_normal_ = nn.init.trunc_normal_
    timm.models = tmod
    tmod.layers = layers
    sys.modules.update({"torchvision": tv, "torchvision.transforms": tv.transforms,
                        "torchvision.utils": tvu, "timm": timm, "timm.models": tmod,
                        "timm.models.layers": layers})
    return load_module("ref_unext", os.path.join(REF, "Experiments/nets/UNext.py")).UNext


def unext(U):
    """7) UNeXt (BASELINE configs[4]; Experiments/nets/UNext.py:201-358), reference-run:
    2x3x64x64 train fwd + WeightedDiceBCE(0.5, 0.5) + bwd (outputs, loss, gradient
    summaries, running-stat sums) and eval output, plus the eval output of one
    1x3x224x224 image (the Cfg5 resolution)."""
    cls = ref_unext(U)
    spec = O.unext_param_spec(3, 1)
    res = {}
    for name, shape, mode in (("s64", (2, 3, 64, 64), "both"), ("s224", (1, 3, 224, 224), "eval")):
        m = cls(num_classes=1, input_channels=3, img_size=shape[-1])
        assert [k for k, _ in spec] == list(m.state_dict().keys())
        sd = O.det_state_dict(spec, seed=5)
        x = O.det_input(shape, f"unext-x-{name}")
        m.load_state_dict(sd)
        m.eval()
        with torch.no_grad():
            res[f"out_eval_{name}"] = m(x).numpy()
        if mode == "both":
            mk = O.det_mask((shape[0], 1) + shape[2:], f"unext-mask-{name}", p=0.3)
            m.load_state_dict(sd)
            m.train()
            out = m(x)
            crit = U.WeightedDiceBCE(dice_weight=0.5, BCE_weight=0.5)
            loss = crit(out, mk.clone())
            m.zero_grad()
            loss.backward()
            names, s1, s2, s3, samp = grad_summary(m)
            bufs = {k: t.detach().numpy() for k, t in m.state_dict().items()
                    if k.endswith("running_mean") or k.endswith("running_var")}
            rm = sorted(bufs)
            res.update({f"out_train_{name}": out.detach().numpy(),
                        f"loss_{name}": np.array(loss.item()), "grad_names": np.array(names),
                        "grad_sum": s1, "grad_abs": s2, "grad_sq": s3, "grad_samples": samp,
                        "buf_names": np.array(rm),
                        "buf_sums": np.array([bufs[k].astype(np.float64).sum() for k in rm])})
            print("unext", name, "loss", loss.item())
    np.savez_compressed(os.path.join(HERE, "unext.npz"), **res)


def grad_summary(model):
    names, s1, s2, s3, samp = [], [], [], [], []
    for n, p in model.named_parameters():
        g = p.grad
        if g is None:
            g = torch.zeros_like(p)
        g = g.detach().double().flatten()
        names.append(n)
        s1.append(g.sum().item())
        s2.append(g.abs().sum().item())
        s3.append((g * g).sum().item())
        idx = torch.linspace(0, g.numel() - 1, 8).long()
        samp.append(g[idx].numpy())
    return names, np.array(s1), np.array(s2), np.array(s3), np.stack(samp)


def fullwidth(models, U):
    """6) The full-width models at the bench resolution (pin n_filts=32 at
    256^2): canonical ACC_UNet (16.77 M, ACC_UNet/ACC_UNet.py:535-659) eval output on
    1x3x256x256, and train-mode fwd + WeightedDiceBCE + bwd on 2x3x256x256 for the
    canonical and the script variant (logits, Experiments/nets/ACC_UNet.py:530-655):
    outputs, loss, per-parameter gradient summaries and running-stat sums."""
    x1 = O.det_input((1, 3, 256, 256), "fw-x1")
    x2 = O.det_input((2, 3, 256, 256), "fw-x2")
    m2 = O.det_mask((2, 1, 256, 256), "fw-mask", p=0.3)
    for v in ("canonical", "script"):
        torch.manual_seed(0)
        m = models[v](3, 1)
        spec = [(k, tuple(t.shape)) for k, t in m.state_dict().items()]
        sd = O.det_state_dict(spec, seed=7)
        res = {}
        if v == "canonical":
            m.load_state_dict(sd)
            m.eval()
            with torch.no_grad():
                res["out_eval"] = m(x1).numpy()
        m.load_state_dict(sd)
        m.train()
        out = m(x2)
        crit = U.WeightedDiceBCE(dice_weight=0.5, BCE_weight=0.5)
        loss = crit(out, m2.clone())
        m.zero_grad()
        loss.backward()
        names, s1, s2, s3, samp = grad_summary(m)
        bufs = {k: t.detach().numpy() for k, t in m.state_dict().items()
                if k.endswith("running_mean") or k.endswith("running_var")}
        rm_names = sorted(bufs)
        np.savez_compressed(
            os.path.join(HERE, f"fullwidth_{v}_nf32.npz"), out_train=out.detach().numpy(),
            loss=np.array(loss.item()), grad_names=np.array(names), grad_sum=s1, grad_abs=s2,
            grad_sq=s3, grad_samples=samp, buf_names=np.array(rm_names),
            buf_sums=np.array([bufs[k].astype(np.float64).sum() for k in rm_names]),
            show_dice=np.array(float(crit._show_dice(out.detach(), m2.clone()))), **res)
        print("fullwidth", v, "loss", loss.item())


def main():
    torch.set_num_threads(8)
    models = ref_models()
    U = ref_utils()
    if "--fullwidth" in sys.argv:
        fullwidth(models, U)
        return
    if "--unext" in sys.argv:
        unext(U)
        return
    meta = {}

    # 1) state_dict key/shape lists at the default size (n_filts=32, n_channels=3) and a
    #    digest of the seeded default initialisation (torch.manual_seed(0); cls(3, 1))
    import hashlib
    for v, cls in models.items():
        torch.manual_seed(0)
        m = cls(3, 1)
        keys = [[k, list(t.shape)] for k, t in m.state_dict().items()]
        nparams = sum(p.numel() for p in m.parameters())
        h = hashlib.sha256()
        for k, t in m.state_dict().items():
            h.update(t.detach().contiguous().numpy().tobytes())
        with open(os.path.join(HERE, f"keys_{v}.json"), "w") as f:
            json.dump({"n_params": nparams, "keys": keys, "init_sha256_seed0": h.hexdigest(),
                       "torch": torch.__version__}, f)
        meta[f"n_params_{v}"] = nparams
        print(v, nparams, len(keys))

    # 2) whole model, n_filts=8, 2x3x32x32, train fwd+loss+bwd and eval fwd
    x = O.det_input((2, 3, 32, 32), "golden-x")
    mask = O.det_mask((2, 1, 32, 32), "golden-mask", p=0.4)
    for v, cls in models.items():
        torch.manual_seed(0)
        m = cls(3, 1, n_filts=8)
        spec = [(k, tuple(t.shape)) for k, t in m.state_dict().items()]
        sd = O.det_state_dict(spec, seed=0)
        m.load_state_dict(sd)
        m.eval()
        with torch.no_grad():
            out_eval = m(x).detach().numpy()
        m.load_state_dict(sd)
        m.train()
        out = m(x)
        crit = U.WeightedDiceBCE(dice_weight=0.5, BCE_weight=0.5)
        loss = crit(out, mask.clone())
        m.zero_grad()
        loss.backward()
        names, s1, s2, s3, samp = grad_summary(m)
        bufs = {k: t.detach().numpy() for k, t in m.state_dict().items()
                if k.endswith("running_mean") or k.endswith("running_var")}
        rm_names = sorted(bufs)
        np.savez_compressed(
            os.path.join(HERE, f"model_{v}_nf8.npz"),
            out_train=out.detach().numpy(), out_eval=out_eval, loss=np.array(loss.item()),
            grad_names=np.array(names), grad_sum=s1, grad_abs=s2, grad_sq=s3, grad_samples=samp,
            buf_names=np.array(rm_names),
            buf_sums=np.array([bufs[k].astype(np.float64).sum() for k in rm_names]),
            show_dice=np.array(float(crit._show_dice(out.detach(), mask.clone()))),
            dice_on_batch=np.array(float(U.dice_on_batch(mask.clone(), out.detach()))),
        )
        print("model", v, "loss", loss.item())

    # 3) Cfg1 plumbing: ACC_UNet_Lite (n_filts 32) forward on 1x3x128x128
    m = models["lite"](3, 1)
    spec = [(k, tuple(t.shape)) for k, t in m.state_dict().items()]
    sd = O.det_state_dict(spec, seed=1)
    xc = O.det_input((1, 3, 128, 128), "cfg1-x")
    mc = O.det_mask((1, 1, 128, 128), "cfg1-mask", p=0.5)
    res = {}
    for mode in ("eval", "train"):
        m.load_state_dict(sd)
        m.train(mode == "train")
        with torch.no_grad():
            o = m(xc)
        crit = U.WeightedDiceBCE(dice_weight=0.5, BCE_weight=0.5)
        res[f"probs_{mode}"] = o.numpy()
        res[f"show_dice_{mode}"] = np.array(float(crit._show_dice(o, mc.clone())))
        res[f"dice_on_batch_{mode}"] = np.array(float(U.dice_on_batch(mc.clone(), o)))
        res[f"loss_{mode}"] = np.array(float(crit(o, mc.clone())))
    np.savez_compressed(os.path.join(HERE, "cfg1_lite.npz"), **res)
    print("cfg1", {k: float(v) for k, v in res.items() if v.ndim == 0})

    # 4) 3-step training trajectory: script variant, n_channels=1, 2x1x64x64, Adam 1e-3
    m = models["script"](1, 1)
    spec = [(k, tuple(t.shape)) for k, t in m.state_dict().items()]
    m.load_state_dict(O.det_state_dict(spec, seed=2))
    m.train()
    opt = torch.optim.Adam(filter(lambda p: p.requires_grad, m.parameters()), lr=1e-3)
    crit = U.WeightedDiceBCE(dice_weight=0.5, BCE_weight=0.5)
    xt = O.det_input((2, 1, 64, 64), "traj-x")
    mt = O.det_mask((2, 1, 64, 64), "traj-mask", p=0.3)
    losses, dices = [], []
    for step in range(3):
        out = m(xt)
        loss = crit(out, mt.clone())
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
        dices.append(float(crit._show_dice(out.detach(), mt.clone())))
    np.savez_compressed(os.path.join(HERE, "traj_script.npz"), losses=np.array(losses),
                        dices=np.array(dices))
    print("traj", losses, dices)

    # 5) cosine warm restarts schedule (T_0=10, eta_min=1e-5), 25 epochs
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=1e-3)
    sch = U.CosineAnnealingWarmRestarts(opt, T_0=10, eta_min=1e-5)
    lrs = []
    for _ in range(25):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    np.savez_compressed(os.path.join(HERE, "lr_schedule.npz"), lrs=np.array(lrs))

    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)

    fullwidth(models, U)
    unext(U)


if __name__ == "__main__":
    main()
