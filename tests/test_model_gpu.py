"""GPU parity: the HIP path (C ABI through the drop-in modules) against the CPU
oracle (fp64) on identical deterministic weights / inputs.

Tolerances (fp32 kernels; the north_star bound is 1e-4 fp32 on outputs / Dice):
  well-conditioned cases (eval mode, single blocks, loss, Adam): absolute bounds
  (probabilities / Dice 1e-4 vs the reference's own outputs, see each test);
  ill-conditioned training-mode BatchNorm over few values (whole model at
  2x3x32x32, Cfg1 train at B = 1): every output / gradient / running statistic
  within 4x the reference's OWN fp32 error (the fp32 oracle runs the same ATen
  ops as the reference) of the fp64 oracle, plus 1e-4 of the tensor's scale.
"""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import parity_util as PU  # noqa: E402
from parity_util import O  # noqa: E402
from accunet import model as M  # noqa: E402
from accunet.loss import WeightedDiceBCE  # noqa: E402
from accunet.optim import FusedAdam  # noqa: E402

DEV = "cuda"
GOLD = os.path.join(HERE, "golden")


def _hip_model(variant, sd, nf, n_ch=3):
    m = M.VARIANTS[variant](n_ch, 1, n_filts=nf)
    m.load_state_dict(sd)
    return m.to(DEV)


@pytest.mark.parametrize("variant", ["canonical", "script", "lite", "w"])
def test_golden_config_loss_and_outputs_match_reference(variant):
    """The golden configuration (n_filts 8, 2x3x32x32): the reference's own fp32
    outputs / loss / Dice (tests/golden/model_*_nf8.npz) vs the HIP path."""
    g = np.load(os.path.join(GOLD, f"model_{variant}_nf8.npz"))
    spec = O.param_spec(variant, 3, 1, 8)
    sd = O.det_state_dict(spec, seed=0)
    x = O.det_input((2, 3, 32, 32), "golden-x")
    mask = O.det_mask((2, 1, 32, 32), "golden-mask", p=0.4)
    m = _hip_model(variant, sd, 8).train()
    crit = WeightedDiceBCE(0.5, 0.5)
    out = m(x.to(DEV))
    loss = crit(out, mask.to(DEV))
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    # 2x2 BatchNorm level: the reference itself is 8e-4 (3e-3 for logits) from fp64
    o64, _, _, _ = PU.oracle_run(variant, sd, x, None)
    e_ref = np.abs(g["out_train"] - o64.numpy()).max()
    e_hip = (out.detach().double().cpu() - o64).abs().max().item()
    assert e_hip <= 4 * e_ref + 1e-5, (e_hip, e_ref)
    # hard masks (sigmoid >= 0.5) may differ only where the reference itself is
    # ambiguous (|sigmoid(out) - 0.5| within its own fp32 error); then Dice within 1e-4
    p_ref = torch.sigmoid(torch.from_numpy(g["out_train"]).double())
    p_hip = torch.sigmoid(out.detach().double().cpu())
    flip = (p_ref >= 0.5) != (p_hip >= 0.5)
    ambiguous = (torch.sigmoid(o64) - 0.5).abs() <= 4 * e_ref + 1e-6
    assert bool((~flip | ambiguous).all())
    if not bool(flip.any()):
        assert abs(crit._show_dice(out.detach(), mask.clone().to(DEV)).item()
                   - float(g["show_dice"])) < 1e-4
        assert abs(O.dice_on_batch(mask.clone(), out.detach().cpu())
                   - float(g["dice_on_batch"])) < 1e-4


@pytest.mark.parametrize("variant", ["canonical", "script", "lite", "w"])
def test_whole_model_train_step_matches_oracle(variant):
    """Full train step (fwd + loss + bwd) at n_filts 8, 4x3x64x64 against the fp64
    oracle, with the reference's OWN fp32 error (fp32 oracle = the reference's ATen
    ops) as the yardstick:
      - whole gradient vector: ||g_hip - g64|| <= 3 ||g32 - g64|| + 1e-6 ||g64||
      - every tensor (outputs, gradients, BN running stats):
          max|hip - 64| <= 4 max|32 - 64| + 1e-4 max|64| + 0.05 * median_k mean|g_k|
        (max|32 - 64| is taken over the reference's fp32 run and two fp32 runs on
        rounding-perturbed inputs/weights; the absolute floor covers near-structurally-zero gradients; SE gate
        fc1 weights/biases, which a batch-wide BatchNorm nearly cancels, get 0.5 * median)
      - loss within 1e-6 relative of the fp64 oracle."""
    nf, B, S = 8, 4, 64
    spec = O.param_spec(variant, 3, 1, nf)
    sd = O.det_state_dict(spec, seed=0)
    x = O.det_input((B, 3, S, S), "golden-x")
    mask = O.det_mask((B, 1, S, S), "golden-mask", p=0.4)
    ref_out, ref_loss, ref_grads, ref_sd = PU.oracle_run(variant, sd, x, mask)
    r32_out, r32_loss, r32_grads, r32_sd = PU.oracle_run(variant, sd, x, mask,
                                                        dtype=torch.float32)
    m = _hip_model(variant, sd, nf).train()
    out = m(x.to(DEV))
    loss = WeightedDiceBCE(0.5, 0.5)(out, mask.to(DEV))
    loss.backward()
    assert abs(loss.item() - ref_loss.item()) <= 1e-6 * abs(ref_loss.item()) + 1e-7
    hip = {"out": out}
    r64 = {"out": ref_out}
    r32 = {"out": r32_out}
    gkeys = []
    for k, p in m.named_parameters():
        hip["grad:" + k] = p.grad if p.grad is not None else torch.zeros_like(p)
        r64["grad:" + k] = ref_grads[k]
        r32["grad:" + k] = r32_grads[k]
        gkeys.append("grad:" + k)
    e_glob_h = PU.global_rel_err(hip, r64, gkeys)
    e_glob_r = PU.global_rel_err(r32, r64, gkeys)
    assert e_glob_h <= 3 * e_glob_r + 1e-6, (e_glob_h, e_glob_r)
    med = PU.median_live_grad(ref_grads)
    # SE gate fc1 (weight and bias): d/d(fc1) = sums over the batch of per-sample terms
    # that the SE's own training BatchNorm (over only B=4 samples here) nearly cancels
    # (a batch-uniform gate shift is normalised away) -> cancellation-dominated; the
    # reference's own fp32 error on them varies ~4x between rounding-perturbed runs
    floor = {k: (0.5 if ".fc1." in k else 0.05) * med for k in gkeys}
    msd = m.state_dict()
    for k, v in ref_sd.items():
        if k.endswith(("running_mean", "running_var")):
            hip["buf:" + k] = msd[k]
            r64["buf:" + k] = v
            r32["buf:" + k] = r32_sd[k]
        elif k.endswith("num_batches_tracked"):
            assert int(msd[k]) == int(v), k
    # fp32 noise of each tensor = max over the reference's fp32 run and two fp32 runs
    # on rounding-perturbed inputs/weights (cancellation-dominated tensors, e.g. BN
    # biases whose gradient the next BatchNorm nearly cancels, swing by several x)
    ens = PU.oracle_run_fp32_ensemble(variant, sd, x, mask)
    rows = PU.compare_vs_reference_fp32(hip, r64, r32, abs_floor=floor, ref32_extra=ens)
    bad = [r for r in rows if not r[4]]
    assert not bad, sorted(bad, key=lambda r: -r[1] / r[3])[:8]
    # and per tensor in norm, with no absolute floor: no gradient may be wrong as a whole
    rows = PU.per_tensor_norm_rows(hip, r64, [r32] + list(ens), gkeys)
    bad = [r for r in rows if not r[4]]
    assert not bad, sorted(bad, key=lambda r: -r[1] / r[3])[:8]
    # eval mode uses the (updated) running statistics
    m.eval()
    with torch.no_grad():
        oe = m(x.to(DEV)).double().cpu()
    ref_e, _, _, _ = PU.oracle_run(variant, ref_sd, x, None, training=False)
    r32_e, _, _, _ = PU.oracle_run(variant, r32_sd, x, None, training=False,
                                   dtype=torch.float32)
    e_h = (oe - ref_e).abs().max().item()
    e_r = (r32_e.double() - ref_e).abs().max().item()
    assert e_h <= 4 * e_r + 1e-5, (e_h, e_r)


def test_cfg1_lite_forward_and_dice_match_reference_golden():
    """BASELINE configs[0]: ACC_UNet_Lite forward on 1x3x128x128 (Dice vs mask).

    eval: probabilities within 1e-4 of the reference's own output (golden), Dice
    within 1e-4. train (B = 1: BatchNorm over 64 values at 8x8): the reference's
    fp32 output itself sits 1.4e-4 from the fp64 oracle, so probabilities are held
    to 4x that distance from the fp64 oracle; Dice still within 1e-4."""
    g = np.load(os.path.join(GOLD, "cfg1_lite.npz"))
    spec = O.param_spec("lite", 3, 1, 32)
    sd0 = O.det_state_dict(spec, seed=1)
    xc = O.det_input((1, 3, 128, 128), "cfg1-x")
    x = xc.to(DEV)
    mk = O.det_mask((1, 1, 128, 128), "cfg1-mask", p=0.5)
    crit = WeightedDiceBCE(0.5, 0.5)
    for mode in ("eval", "train"):
        m = _hip_model("lite", sd0, 32).train(mode == "train")
        with torch.no_grad():
            probs = m(x)
        p = probs.double().cpu()
        if mode == "eval":
            d = np.abs(p.numpy() - g["probs_eval"]).max()
            assert d < 1e-4, (mode, d)
        else:
            with torch.no_grad():
                o64, _, _, _ = PU.oracle_run("lite", sd0, xc, None, training=True)
            e_ref = np.abs(g["probs_train"] - o64.numpy()).max()
            e_hip = (p - o64).abs().max().item()
            assert e_hip <= 4 * e_ref + 1e-5, (e_hip, e_ref)
        sd = crit._show_dice(probs, mk.clone().to(DEV)).item()
        assert abs(sd - float(g[f"show_dice_{mode}"])) < 1e-4
        assert abs(O.dice_on_batch(mk.clone(), probs.cpu()) - float(g[f"dice_on_batch_{mode}"])) < 1e-4
        assert abs(crit(probs, mk.to(DEV)).item() - float(g[f"loss_{mode}"])) < 1e-5


def test_training_trajectory_matches_reference_golden():
    """3 Adam steps of the script variant (n_channels 1, 2x1x64x64) vs the reference."""
    g = np.load(os.path.join(GOLD, "traj_script.npz"))
    spec = O.param_spec("script", 1, 1, 32)
    sd = O.det_state_dict(spec, seed=2)
    m = _hip_model("script", sd, 32, n_ch=1).train()
    opt = FusedAdam([p for p in m.parameters() if p.requires_grad], lr=1e-3)
    crit = WeightedDiceBCE(0.5, 0.5)
    x = O.det_input((2, 1, 64, 64), "traj-x").to(DEV)
    mk = O.det_mask((2, 1, 64, 64), "traj-mask", p=0.3).to(DEV)
    losses = []
    for _ in range(3):
        out = m(x)
        loss = crit(out, mk)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    # Adam divides every gradient by its own RMS, so parameters whose true gradient is
    # ~0 take lr-sized steps along their rounding noise: even the fp64 oracle departs
    # from the reference's fp32 trajectory by 1.6e-3 at step 2 (1.8e-3 at step 3).
    # Step 1 (no update yet) is pinned tightly, later steps to that inherent spread.
    assert abs(losses[0] - g["losses"][0]) < 1e-5, (losses, list(g["losses"]))
    assert abs(losses[1] - g["losses"][1]) < 4e-3, (losses, list(g["losses"]))
    assert abs(losses[2] - g["losses"][2]) < 1e-2, (losses, list(g["losses"]))
    assert losses[2] < losses[0]  # it trains


def test_fused_adam_matches_torch_adam():
    torch.manual_seed(0)
    ps = [torch.randn(s, device=DEV) for s in ((300, 7), (5,), (40000,))]
    qs = [p.clone() for p in ps]
    pa = [torch.nn.Parameter(p) for p in ps]
    pb = [torch.nn.Parameter(q) for q in qs]
    oa = FusedAdam(pa, lr=1e-3)
    ob = torch.optim.Adam(pb, lr=1e-3, foreach=False)
    for it in range(4):
        for a, b in zip(pa, pb):
            gr = torch.randn_like(a) * (it + 1)
            a.grad = gr.clone()
            b.grad = gr.clone()
        oa.step()
        ob.step()
    for a, b in zip(pa, pb):
        assert (a - b).abs().max().item() < 1e-6


def test_loss_matches_oracle_including_binarised_masks():
    torch.manual_seed(3)
    x = torch.randn(3, 1, 16, 16, dtype=torch.float64)
    for scale in (1.0, 255.0):
        t = (torch.rand(3, 1, 16, 16) < 0.3).double() * scale
        xr = x.clone().requires_grad_(True)
        lr = O.dice_bce_loss(xr, t)
        lr.backward()
        xh = x.float().to(DEV).requires_grad_(True)
        lh = WeightedDiceBCE(0.5, 0.5)(xh, t.float().to(DEV))
        lh.backward()
        assert abs(lh.item() - lr.item()) < 1e-5
        assert (xh.grad.double().cpu() - xr.grad).abs().max().item() < 1e-6


@pytest.mark.parametrize("k,cin,cout", [(1, 16, 32), (2, 8, 16), (3, 8, 8), (3, 3, 16)])
def test_hanc_block_matches_oracle(k, cin, cout):
    torch.manual_seed(0)
    blk = M.HANCBlock(cin, cout, k=k, inv_fctr=3)
    spec = [(n, tuple(t.shape)) for n, t in blk.state_dict().items()]
    sd = O.det_state_dict(spec, seed=5)
    blk.load_state_dict(sd)
    blk = blk.to(DEV).train()
    x = O.det_input((2, cin, 16, 16), f"hb{k}")
    xh = x.to(DEV).requires_grad_(True)
    out = blk(xh)
    go = O.det_input(tuple(out.shape), "hb-go").to(DEV)
    (out * go).sum().backward()
    sdo = {n: (v.double().requires_grad_(not n.endswith(PU.BUFFER_LEAVES)) if v.is_floating_point() else v)
           for n, v in sd.items()}
    # oracle names are prefixed by the block path; bind through a prefix-less dict
    xr = x.double().requires_grad_(True)
    ref = O.hanc_block(xr, {("b." + n): v for n, v in sdo.items()}, "b", k, True)
    (ref * go.double().cpu()).sum().backward()
    assert (out.detach().double().cpu() - ref.detach()).abs().max().item() < 1e-4
    assert (xh.grad.double().cpu() - xr.grad).abs().max().item() < 1e-4 * max(1.0, xr.grad.abs().max().item())
    for n, p in blk.named_parameters():
        gr = sdo[n].grad
        if gr is None or PU.structurally_zero("x." + n):
            continue
        err = (p.grad.double().cpu() - gr).abs().max().item()
        assert err < 2e-3 * gr.abs().max().item() + 1e-6, n


def test_maxpool_first_max_tie_rule():
    x = torch.zeros(1, 4, 4, 8, device=DEV)  # all ties: gradient goes to the top-left element
    from accunet import ops
    xr = x.clone().requires_grad_(True)
    y = ops.pool2(xr)
    y.sum().backward()
    g = xr.grad[0, :, :, 0].cpu()
    assert g[0, 0] == 1 and g[0, 1] == 0 and g[1, 0] == 0 and g[1, 1] == 0


@pytest.mark.parametrize("variant", ["canonical", "lite"])
def test_hip_graph_train_step_equals_eager(variant):
    """bench.py's mode: forward + loss + backward captured once into a HIP graph and
    replayed, then the fused Adam launch. Every kernel is deterministic (no float
    atomics), so 3 graph steps must reproduce 3 eager steps bit for bit: losses,
    parameters, BatchNorm running statistics and num_batches_tracked. The graph step
    reads the forward-layout weight copies of the one-launch WeightPrep (remade before
    every replay from the weights Adam left) and makes the backward's inverse weight
    relayouts in one launch at the end of the backward (ops.DeferredRelayouts); the
    eager step makes both per op."""
    from accunet.train import TrainStep
    nf, B, S = 8, 2, 64
    sd = O.det_state_dict(O.param_spec(variant, 3, 1, nf), seed=0)
    x = O.det_input((B, 3, S, S), "golden-x").to(DEV)
    mask = O.det_mask((B, 1, S, S), "golden-mask", p=0.4).to(DEV)
    runs = {}
    for graph in (False, True):
        m = _hip_model(variant, sd, nf).train()
        step = TrainStep(m, lr=1e-3, graph=graph)
        losses = [float(step(x, mask).item()) for _ in range(3)]
        runs[graph] = (losses, {k: v.detach().clone() for k, v in m.state_dict().items()})
    assert runs[False][0] == runs[True][0], (runs[False][0], runs[True][0])
    for k, v in runs[False][1].items():
        assert torch.equal(v, runs[True][1][k]), k


@pytest.mark.parametrize("graph,precision", [(False, "fp32"), (True, "fp32"), (True, "bf16")])
def test_side_stream_weight_gradients_bit_identical(graph, precision):
    """The weight-gradient GEMMs run on a side stream, concurrently with the data
    gradients (ops._WgradFork; fork / join become graph edges under capture). Two
    training steps with and without the side stream: identical losses, parameters
    and BatchNorm state bit for bit (eager and HIP-graph, fp32 and bf16)."""
    from accunet import ops
    from accunet.train import TrainStep
    nf, B, S = 8, 2, 64
    sd = O.det_state_dict(O.param_spec("canonical", 3, 1, nf), seed=0)
    x = O.det_input((B, 3, S, S), "golden-x").to(DEV)
    mask = O.det_mask((B, 1, S, S), "golden-mask", p=0.4).to(DEV)
    runs = {}
    prev = ops.set_wgrad_stream(True)
    try:
        for side in (False, True):
            ops.set_wgrad_stream(side)
            m = _hip_model("canonical", sd, nf).train()
            step = TrainStep(m, lr=1e-3, graph=graph, precision=precision)
            losses = [float(step(x, mask).item()) for _ in range(2)]
            runs[side] = (losses, {k: v.detach().clone() for k, v in m.state_dict().items()})
    finally:
        ops.set_wgrad_stream(prev)
    assert runs[False][0] == runs[True][0], (runs[False][0], runs[True][0])
    for k, v in runs[False][1].items():
        assert torch.equal(v, runs[True][1][k]), k


@pytest.mark.parametrize("variant", ["canonical", "script", "lite", "w"])
def test_eval_mode_backward_matches_oracle(variant):
    """Backward with the BatchNorms on their running statistics (model.eval(), as when a
    caller fine-tunes or probes gradients of the reference module in eval mode): every
    parameter gradient of the fp32 HIP path within 4x the fp32 oracle's own error of
    the fp64 oracle, the whole gradient within 3x its relative error, same direction."""
    nf, B, S = 8, 2, 32
    sd = O.det_state_dict(O.param_spec(variant, 3, 1, nf), seed=0)
    x = O.det_input((B, 3, S, S), "golden-x")
    mask = O.det_mask((B, 1, S, S), "golden-mask", p=0.4)
    o64, l64, g64, _ = PU.oracle_run(variant, sd, x, mask, training=False)
    o32, l32, g32, _ = PU.oracle_run(variant, sd, x, mask, dtype=torch.float32, training=False)
    m = _hip_model(variant, sd, nf).eval()
    out = m(x.to(DEV))
    loss = WeightedDiceBCE(0.5, 0.5)(out, mask.to(DEV))
    loss.backward()
    keys = [k for k, _ in m.named_parameters()]
    hip = {k: (p.grad if p.grad is not None else torch.zeros_like(p)) for k, p in m.named_parameters()}
    for k in keys:
        ref = g64[k]
        e32 = (g32[k].double() - ref).abs().max().item()
        eh = (hip[k].double().cpu() - ref).abs().max().item()
        assert eh <= 4 * e32 + 1e-4 * ref.abs().max().item() + 1e-9, (k, eh, e32)
    eg_h = PU.global_rel_err(hip, g64, keys)
    eg_32 = PU.global_rel_err(g32, g64, keys)
    assert eg_h <= 3 * eg_32 + 1e-6, (eg_h, eg_32)
    assert PU.grad_cosine(hip, g64, keys) >= 1 - 1e-9
    assert abs(loss.item() - l64.item()) <= 4 * abs(l32.item() - l64.item()) + 1e-6
    assert (out.double().cpu() - o64).abs().max().item() < 1e-4


@pytest.mark.parametrize("graph", [False, True])
def test_selective_fork_bit_identical(graph):
    """ACCUNET_WGRAD_FORK_MIN_US > 0 (ops.set_wgrad_fork_min_us): some layers' weight
    gradients run on the side stream and the others on the main stream in the same
    backward. Two training steps at cuts 0 (fork every layer), the median of the
    estimates the first run logged (a mix) and 1e9 (never fork): identical losses,
    parameters and BatchNorm state bit for bit."""
    from accunet import ops
    from accunet.train import TrainStep
    nf, B, S = 32, 4, 64
    sd = O.det_state_dict(O.param_spec("canonical", 3, 1, nf), seed=0)
    x = O.det_input((B, 3, S, S), "golden-x").to(DEV)
    mask = O.det_mask((B, 1, S, S), "golden-mask", p=0.4).to(DEV)
    runs = {}
    prev_s = ops.set_wgrad_stream(True)
    prev_c = ops.set_wgrad_fork_min_us(0.0)
    try:
        ops.FORK_LOG = []
        cuts = [0.0, None, 1e9]
        for i, cut in enumerate(cuts):
            if cut is None:  # the median estimate of the first run splits the layers
                est = sorted(ops.FORK_LOG)
                cut = cuts[i] = est[len(est) // 2] + 1e-9
            ops.set_wgrad_fork_min_us(cut)
            m = _hip_model("canonical", sd, nf).train()
            step = TrainStep(m, lr=1e-3, graph=graph)
            c0 = list(ops.FORK_COUNTS)
            losses = [float(step(x, mask).item()) for _ in range(2)]
            kept, forked = (ops.FORK_COUNTS[0] - c0[0], ops.FORK_COUNTS[1] - c0[1])
            if i == 1:  # the mixed configuration really mixes
                assert kept > 0 and forked > 0, (cut, kept, forked)
            runs[cut] = (losses, {k: v.detach().clone() for k, v in m.state_dict().items()})
    finally:
        ops.FORK_LOG = None
        ops.set_wgrad_stream(prev_s)
        ops.set_wgrad_fork_min_us(prev_c)
    for cut in cuts[1:]:
        assert runs[0.0][0] == runs[cut][0], (cut, runs[0.0][0], runs[cut][0])
        for k, v in runs[0.0][1].items():
            assert torch.equal(v, runs[cut][1][k]), (cut, k)


@pytest.mark.parametrize("variant,B,S", [("canonical", 16, 256), ("w", 4, 512)])
def test_full_size_configs_properties(variant, B, S):
    """BASELINE configs[1] (canonical, 16x3x256x256) and configs[3] (ACC_UNet_W,
    4x3x512x512) at full size, where the fp64 oracle is too slow to run: properties
    that hold at any size. (1) determinism: two training steps from the same state
    are bit-identical (no float atomics anywhere); (2) probabilities in [0, 1] and
    every gradient finite; (3) the loss of the HIP forward equals WeightedDiceBCE
    recomputed in fp64 from the HIP probabilities (loss kernel at full size);
    (4) three Adam steps on one batch lower the loss."""
    from accunet.train import TrainStep
    torch.manual_seed(0)
    m = M.VARIANTS[variant](3, 1, n_filts=32).to(DEV).train()
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, 3, S, S, generator=g).to(DEV)
    mask = (torch.rand(B, 1, S, S, generator=g) < 0.3).float().to(DEV)
    crit = WeightedDiceBCE(0.5, 0.5)
    grads = []
    for _ in range(2):
        m.load_state_dict(sd0)
        m.zero_grad(set_to_none=True)
        out = m(x)
        loss = crit(out, mask)
        loss.backward()
        grads.append((out.detach().clone(), float(loss),
                      [p.grad.detach().clone() for p in m.parameters() if p.grad is not None]))
    (o1, l1, g1), (o2, l2, g2) = grads
    assert torch.equal(o1, o2) and l1 == l2
    assert all(torch.equal(a, b) for a, b in zip(g1, g2))
    assert float(o1.min()) >= 0.0 and float(o1.max()) <= 1.0
    assert all(torch.isfinite(a).all() for a in g1)
    ref = O.dice_bce_loss(o1.double().cpu(), mask.double().cpu())
    assert abs(l1 - float(ref)) < 1e-5 * max(1.0, abs(float(ref)))
    m.load_state_dict(sd0)
    step = TrainStep(m, lr=1e-3, graph=False)
    losses = [float(step(x, mask)) for _ in range(4)]
    assert losses[-1] < losses[0], losses


@pytest.mark.parametrize("variant", ["canonical", "script"])
def test_fullwidth_nf32_at_256_matches_reference_and_oracle(variant):
    """The bench-width models (n_filts 32; canonical = 16.77 M with cnv72 inv_fctr 34)
    at 256^2, where every shape-gated kernel path of the bench runs (K <= 64 small-K
    tiles over M >= 65536 pixels with the pyramid / BN-backward epilogues, the
    skinny weight-gradient path, the < 128-tile rule at 16^2):
      - train fwd + WeightedDiceBCE + bwd on 2x3x256x256 against the reference's own
        fp32 run (tests/golden/fullwidth_*_nf32.npz, made by importing the
        reference) and the fp64 oracle: output within 4x the reference's own fp32
        distance to fp64 + 1e-4 of scale, loss within 1e-5 of the reference's;
      - every gradient and running statistic within 4x the fp32 distance to fp64,
        taken as the max over the fp32 oracle run and an ensemble of fp32 runs on
        2^-24-perturbed inputs (parity_util.oracle_run_fp32_ensemble: one fp32 run
        under-states the sensitivity of cancellation-dominated tensors several x, e.g.
        cnv11.norm1.weight 2.8e-4 single vs 9.3e-4 ensemble; tools/fw_diag.py), plus
        the floors of test_whole_model_train_step_matches_oracle, every gradient in norm
        within 4x the ensemble's norm distance with no floor, and the whole gradient
        vector within 3x of the single run;
      - canonical eval output on 1x3x256x256 within 1e-4 of the reference's (the
        north-star bound)."""
    g = np.load(os.path.join(GOLD, f"fullwidth_{variant}_nf32.npz"))
    spec = O.param_spec(variant, 3, 1, 32)
    sd = O.det_state_dict(spec, seed=7)
    torch.set_num_threads(16)
    if variant == "canonical":
        m = _hip_model(variant, sd, 32).eval()
        with torch.no_grad():
            oe = m(O.det_input((1, 3, 256, 256), "fw-x1").to(DEV)).double().cpu().numpy()
        assert np.abs(oe - g["out_eval"]).max() < 1e-4
        del m
    x = O.det_input((2, 3, 256, 256), "fw-x2")
    mask = O.det_mask((2, 1, 256, 256), "fw-mask", p=0.3)
    m = _hip_model(variant, sd, 32).train()
    out = m(x.to(DEV))
    loss = WeightedDiceBCE(0.5, 0.5)(out, mask.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - float(g["loss"])) < 1e-5, (loss.item(), float(g["loss"]))
    ref_out, ref_loss, ref_grads, ref_sd = PU.oracle_run(variant, sd, x, mask)
    e_ref = float(np.abs(g["out_train"] - ref_out.numpy()).max())
    e_hip = (out.detach().double().cpu() - ref_out).abs().max().item()
    assert e_hip <= 4 * e_ref + 1e-4 * ref_out.abs().max().item(), (e_hip, e_ref)
    r32_out, _, r32_grads, r32_sd = PU.oracle_run(variant, sd, x, mask, dtype=torch.float32)
    hip, r64, r32 = {"out": out}, {"out": ref_out}, {"out": r32_out}
    gkeys = []
    for k, p in m.named_parameters():
        hip["grad:" + k] = p.grad if p.grad is not None else torch.zeros_like(p)
        r64["grad:" + k] = ref_grads[k]
        r32["grad:" + k] = r32_grads[k]
        gkeys.append("grad:" + k)
    e_glob_h = PU.global_rel_err(hip, r64, gkeys)
    e_glob_r = PU.global_rel_err(r32, r64, gkeys)
    assert e_glob_h <= 3 * e_glob_r + 1e-6, (e_glob_h, e_glob_r)
    med = PU.median_live_grad(ref_grads)
    floor = {k: (0.5 if ".fc1." in k else 0.05) * med for k in gkeys}
    msd = m.state_dict()
    for k, v in ref_sd.items():
        if k.endswith(("running_mean", "running_var")):
            hip["buf:" + k] = msd[k]
            r64["buf:" + k] = v
            r32["buf:" + k] = r32_sd[k]
    ens = PU.oracle_run_fp32_ensemble(variant, sd, x, mask)
    rows = PU.compare_vs_reference_fp32(hip, r64, r32, abs_floor=floor, ref32_extra=ens)
    bad = [r for r in rows if not r[4]]
    assert not bad, sorted(bad, key=lambda r: -r[1] / r[3])[:8]
    # and per tensor in norm, with no absolute floor (the bench-width tile rules and the
    # 32-channel halo convolutions run only at this width): no gradient wrong as a whole
    rows = PU.per_tensor_norm_rows(hip, r64, [r32] + list(ens), gkeys)
    bad = [r for r in rows if not r[4]]
    assert not bad, sorted(bad, key=lambda r: -r[1] / r[3])[:8]


def test_multiclass_head_matches_oracle():
    """n_classes > 1 (ACC_UNet/ACC_UNet.py:597-599): n_classes + 1 output channels from
    the 1x1 head, no activation. Train-mode forward and the gradients of a fixed
    linear functional of the output against the fp64 oracle (fp32-error yardstick)."""
    nf, B, S, nc = 8, 2, 32, 2
    spec = O.param_spec("canonical", 3, nc, nf)
    sd = O.det_state_dict(spec, seed=3)
    x = O.det_input((B, 3, S, S), "mc-x")
    go = O.det_input((B, nc + 1, S, S), "mc-go")
    m = M.ACC_UNet(3, nc, n_filts=nf)
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    out = m(x.to(DEV))
    assert tuple(out.shape) == (B, nc + 1, S, S) and m.last_activation is None
    (out * go.to(DEV)).sum().backward()
    res = {}
    for dt in (torch.float64, torch.float32):
        sdo = {k: (v.clone().to(dt).requires_grad_(not k.endswith(PU.BUFFER_LEAVES))
                   if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        o = O.forward(sdo, x.to(dt), "canonical", training=True, n_classes=nc)
        (o * go.to(dt)).sum().backward()
        res[dt] = (o.detach(), {k: v.grad for k, v in sdo.items() if v.is_floating_point()
                                and not k.endswith(PU.BUFFER_LEAVES)})
    (o64, g64), (o32, g32) = res[torch.float64], res[torch.float32]
    e_h = (out.detach().double().cpu() - o64).abs().max().item()
    e_r = (o32.double() - o64).abs().max().item()
    assert e_h <= 4 * e_r + 1e-4 * o64.abs().max().item(), (e_h, e_r)
    hip = {k: p.grad for k, p in m.named_parameters()}
    for k in ("out.weight", "out.bias", "cnv92.conv3.weight", "cnv11.conv1.weight"):
        eh = (hip[k].double().cpu() - g64[k]).abs().max().item()
        er = (g32[k].double() - g64[k]).abs().max().item()
        assert eh <= 4 * er + 1e-4 * g64[k].abs().max().item(), (k, eh, er)
    gk = [k for k in g64 if hip.get(k) is not None]
    num = sum(float((hip[k].double().cpu() - g64[k]).norm() ** 2) for k in gk)
    num32 = sum(float((g32[k].double() - g64[k]).norm() ** 2) for k in gk)
    assert num ** 0.5 <= 3 * num32 ** 0.5 + 1e-9, (num ** 0.5, num32 ** 0.5)
