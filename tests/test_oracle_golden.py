"""Pin the CPU oracle (oracle/accunet_oracle.py) to the reference's own outputs.

The fixtures in tests/golden/ were produced by tests/golden/make_golden.py, which
imports the reference modules in the build container. CPU only.
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import accunet_oracle as O  # noqa: E402

BUFFER_LEAVES = ("running_mean", "running_var", "num_batches_tracked")
# biases of convolutions that feed a training-mode BatchNorm directly: their true
# gradient is exactly 0 (the batch mean removes them); both sides hold rounding noise
BN_FED_BIAS = (".conv1.bias", ".conv2.bias", ".hnc.cnv.bias", ".conv3.bias", ".norm.bias")


def is_bn_fed_bias(name):
    if name.startswith("rspth") and ".convs." in name and name.endswith(".bias"):
        return True
    return name.endswith(BN_FED_BIAS)


def oracle_params(sd):
    params = {}
    for k, v in sd.items():
        if not k.endswith(BUFFER_LEAVES):
            v.requires_grad_(True)
            params[k] = v
    return params


@pytest.mark.parametrize("variant", O.VARIANTS)
def test_state_dict_keys_match_reference(variant):
    with open(os.path.join(GOLD, f"keys_{variant}.json")) as f:
        ref = json.load(f)
    spec = O.param_spec(variant, 3, 1, 32)
    assert [[k, list(s)] for k, s in spec] == ref["keys"]
    n = sum(int(np.prod(s)) for k, s in spec if not k.endswith(BUFFER_LEAVES))
    assert n == ref["n_params"]


def check_grad_summary(params, g, rtol=2e-3, se_rtol=2e-2):
    """The oracle's parameter gradients against the reference's per-tensor summaries
    (sum |g|, 8 samples) written by make_golden.grad_summary. SE gate fc1 gradients
    are sums of per-sample terms that the SE's own batch BatchNorm nearly cancels
    (few samples), so their fp32 op-order noise is ~10x larger: se_rtol."""
    names = list(g["grad_names"])
    assert names == [k for k in params]
    # model-wide gradient scale: median per-element mean |g|; absolute floors are
    # expressed relative to it (SE/BN gradients cancel heavily and carry rounding noise)
    numels = np.array([params[n].numel() for n in names])
    per = g["grad_abs"] / numels
    live = [per[i] for i, n in enumerate(names) if per[i] > 0 and not is_bn_fed_bias(n)]
    med = float(np.median(live))
    floor = 5e-4 * med
    for i, n in enumerate(names):
        gr = params[n].grad
        gr = torch.zeros_like(params[n]) if gr is None else gr
        gr = gr.detach().double().flatten()
        ref_abs = float(g["grad_abs"][i])
        if is_bn_fed_bias(n) or ref_abs / gr.numel() < 1e-4 * med:
            # structurally zero gradient (a following training-mode BatchNorm removes
            # any per-channel constant): only rounding noise on both sides
            assert gr.abs().mean().item() < 0.3 * med and ref_abs / gr.numel() < 0.3 * med, n
            continue
        # sums of |g| and g^2 are robust; the plain sum can cancel to ~0
        # (rtol 2e-3 plus the absolute floor per element)
        rt = se_rtol if ".fc1." in n else rtol
        assert abs(gr.abs().sum().item() - ref_abs) <= rt * ref_abs + floor * gr.numel(), n
        idx = torch.linspace(0, gr.numel() - 1, 8).long()
        scale = gr.abs().max().item()
        np.testing.assert_allclose(gr[idx].numpy(), g["grad_samples"][i],
                                   rtol=0, atol=rt * scale + floor, err_msg=n)


@pytest.mark.parametrize("variant", O.VARIANTS)
def test_whole_model_nf8_matches_reference(variant):
    g = np.load(os.path.join(GOLD, f"model_{variant}_nf8.npz"))
    spec = O.param_spec(variant, 3, 1, 8)
    x = O.det_input((2, 3, 32, 32), "golden-x")
    mask = O.det_mask((2, 1, 32, 32), "golden-mask", p=0.4)
    sd = O.det_state_dict(spec, seed=0)
    with torch.no_grad():
        out_eval = O.forward({k: v.clone() for k, v in sd.items()}, x, variant, training=False)
    np.testing.assert_allclose(out_eval.numpy(), g["out_eval"], rtol=0, atol=2e-5)

    params = oracle_params(sd)
    out = O.forward(sd, x, variant, training=True)
    np.testing.assert_allclose(out.detach().numpy(), g["out_train"], rtol=0, atol=2e-5)
    loss = O.dice_bce_loss(out, mask.clone())
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    loss.backward()
    check_grad_summary(params, g)
    bnames = list(g["buf_names"])
    for i, n in enumerate(bnames):
        assert abs(sd[n].double().sum().item() - float(g["buf_sums"][i])) < 1e-4, n
    sdice = O.show_dice(out.detach(), mask.clone()).item()
    assert abs(sdice - float(g["show_dice"])) < 1e-6
    assert abs(O.dice_on_batch(mask.clone(), out.detach()) - float(g["dice_on_batch"])) < 1e-6


def test_cfg1_lite_matches_reference():
    g = np.load(os.path.join(GOLD, "cfg1_lite.npz"))
    spec = O.param_spec("lite", 3, 1, 32)
    sd0 = O.det_state_dict(spec, seed=1)
    x = O.det_input((1, 3, 128, 128), "cfg1-x")
    m = O.det_mask((1, 1, 128, 128), "cfg1-mask", p=0.5)
    for mode in ("eval", "train"):
        sd = {k: v.clone() for k, v in sd0.items()}
        with torch.no_grad():
            probs = O.forward(sd, x, "lite", training=(mode == "train"))
        np.testing.assert_allclose(probs.numpy(), g[f"probs_{mode}"], rtol=0, atol=1e-5)
        assert abs(O.show_dice(probs, m.clone()).item() - float(g[f"show_dice_{mode}"])) < 1e-6
        assert abs(O.dice_on_batch(m.clone(), probs) - float(g[f"dice_on_batch_{mode}"])) < 1e-6
        assert abs(O.dice_bce_loss(probs, m.clone()).item() - float(g[f"loss_{mode}"])) < 1e-5


def test_training_trajectory_matches_reference():
    g = np.load(os.path.join(GOLD, "traj_script.npz"))
    spec = O.param_spec("script", 1, 1, 32)
    sd = O.det_state_dict(spec, seed=2)
    params = oracle_params(sd)
    opt = torch.optim.Adam(list(params.values()), lr=1e-3)
    x = O.det_input((2, 1, 64, 64), "traj-x")
    m = O.det_mask((2, 1, 64, 64), "traj-mask", p=0.3)
    losses = []
    for _ in range(3):
        out = O.forward(sd, x, "script", training=True)
        loss = O.dice_bce_loss(out, m.clone())
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    # Adam divides each gradient by its own running RMS, so parameters whose true
    # gradient is ~0 (BN-fed biases, SE gates under a batch BN) take lr-sized steps in
    # the direction of their rounding noise: two correct implementations drift apart
    # after the first update. Steps 1-2 are pinned tightly, step 3 loosely.
    np.testing.assert_allclose(losses[:2], g["losses"][:2], rtol=0, atol=2e-5)
    np.testing.assert_allclose(losses[2], g["losses"][2], rtol=0, atol=1e-2)


def test_lr_schedule_matches_reference():
    g = np.load(os.path.join(GOLD, "lr_schedule.npz"))
    lrs = [O.cosine_warm_restarts_lr(1e-3, 1e-5, 10, e) for e in range(25)]
    np.testing.assert_allclose(lrs, g["lrs"], rtol=1e-9)


@pytest.mark.parametrize("variant", ["canonical", "script"])
def test_fullwidth_nf32_at_256_matches_reference(variant):
    """The full-width models (n_filts 32; canonical 16.77 M with cnv72 inv_fctr 34,
    ACC_UNet/ACC_UNet.py:584) at the bench resolution: train fwd + loss + bwd on
    2x3x256x256 (and the canonical eval output on 1x3x256x256) against the reference's
    own fp32 run (tests/golden/fullwidth_*_nf32.npz)."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = np.load(os.path.join(GOLD, f"fullwidth_{variant}_nf32.npz"))
    spec = O.param_spec(variant, 3, 1, 32)
    sd = O.det_state_dict(spec, seed=7)
    if variant == "canonical":
        with torch.no_grad():
            oe = O.forward({k: v.clone() for k, v in sd.items()},
                           O.det_input((1, 3, 256, 256), "fw-x1"), variant, training=False)
        np.testing.assert_allclose(oe.numpy(), g["out_eval"], rtol=0, atol=2e-5)
    x = O.det_input((2, 3, 256, 256), "fw-x2")
    mask = O.det_mask((2, 1, 256, 256), "fw-mask", p=0.3)
    params = oracle_params(sd)
    out = O.forward(sd, x, variant, training=True)
    scale = float(np.abs(g["out_train"]).max())
    np.testing.assert_allclose(out.detach().numpy(), g["out_train"], rtol=0, atol=2e-5 * max(1.0, scale))
    loss = O.dice_bce_loss(out, mask.clone())
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    loss.backward()
    check_grad_summary(params, g)
    for i, n in enumerate(list(g["buf_names"])):
        assert abs(sd[n].double().sum().item() - float(g["buf_sums"][i])) < 1e-4 * max(1.0, abs(float(g["buf_sums"][i]))), n
    assert abs(O.show_dice(out.detach(), mask.clone()).item() - float(g["show_dice"])) < 1e-6


def test_unext_matches_reference():
    """UNeXt (BASELINE configs[4], Experiments/nets/UNext.py:201-358): the oracle's
    restatement (oracle/accunet_oracle.py: unext_forward) against the reference module
    itself, run by tests/golden/make_golden.py with import shims for the absent timm /
    torchvision (to_2tuple restated, trunc_normal_ = torch's, DropPath never built at
    drop_path_rate 0): 2x3x64x64 train fwd + WeightedDiceBCE + bwd (output, loss, every
    parameter gradient's summary, running statistics) and eval outputs at 64^2 and at
    the Cfg5 resolution 224^2 (tests/golden/unext.npz)."""
    g = np.load(os.path.join(GOLD, "unext.npz"))
    spec = O.unext_param_spec(3, 1)
    sd0 = O.det_state_dict(spec, seed=5)
    for name, shape in (("s64", (2, 3, 64, 64)), ("s224", (1, 3, 224, 224))):
        x = O.det_input(shape, f"unext-x-{name}")
        with torch.no_grad():
            oe = O.unext_forward({k: v.clone() for k, v in sd0.items()}, x, training=False)
        np.testing.assert_allclose(oe.numpy(), g[f"out_eval_{name}"], rtol=0, atol=2e-5)
    sd = {k: v.clone() for k, v in sd0.items()}
    x = O.det_input((2, 3, 64, 64), "unext-x-s64")
    mask = O.det_mask((2, 1, 64, 64), "unext-mask-s64", p=0.3)
    params = oracle_params(sd)
    out = O.unext_forward(sd, x, training=True)
    np.testing.assert_allclose(out.detach().numpy(), g["out_train_s64"], rtol=0, atol=2e-5)
    loss = O.dice_bce_loss(out, mask.clone())
    assert abs(loss.item() - float(g["loss_s64"])) < 1e-5
    loss.backward()
    # the encoder / decoder conv biases feed a training-mode BatchNorm (UNext.py:257-330):
    # structurally zero gradients, rounding noise on both sides
    bn_fed = {f"encoder{i}.bias" for i in (1, 2, 3)} | {f"decoder{i}.bias" for i in (1, 2, 3, 4)}
    names = list(g["grad_names"])
    assert names == list(params)
    per = g["grad_abs"] / np.array([params[n].numel() for n in names])
    med = float(np.median(per[per > 0]))
    for i, n in enumerate(names):
        gr = params[n].grad.detach().double().flatten()
        if n in bn_fed:
            assert gr.abs().mean().item() < 1e-3 * med and per[i] < 1e-3 * med, n
            continue
        ref = float(g["grad_abs"][i])
        assert abs(gr.abs().sum().item() - ref) <= 2e-3 * ref + 1e-4 * med * gr.numel(), n
        idx = torch.linspace(0, gr.numel() - 1, 8).long()
        np.testing.assert_allclose(gr[idx].numpy(), g["grad_samples"][i], rtol=0,
                                   atol=2e-3 * gr.abs().max().item() + 1e-4 * med, err_msg=n)
    for i, n in enumerate(list(g["buf_names"])):
        assert abs(sd[n].double().sum().item() - float(g["buf_sums"][i])) < 1e-4, n
