"""bf16 activation mode (BASELINE configs[2]: bf16 activations, fp32 master weights,
fp32 Adam state, fp32 / fp64 BatchNorm and SE statistics) on the GPU.

1. The bf16 GEMM engine (csrc/gemm_bf16.h, v_mfma_f32_32x32x16_bf16) in every operand
   mode against an fp64 product of the SAME bf16-rounded operands: the only
   differences left are fp32 accumulation order and the final rounding of a bf16 C,
   so C is held to half a bf16 ulp of |C| plus the fp32 accumulation error.
2. The whole model trained in bf16 against the fp64 oracle. The yardstick is the
   oracle run in fp64 with bf16 storage rounding emulated at the tensors the build
   stores in bf16 (oracle.storage_rounding): that run's distance to the plain fp64
   oracle is the error bf16 storage alone causes; the HIP bf16 result must be within
   a small factor of it (outputs: 2x mean / 4x max distance; loss: 4x the largest
   of an ensemble of emulated runs; whole gradient vector and BatchNorm running
   statistics: 2x).
3. Bench-size properties (16x3x256x256): determinism, finite gradients, the loss
   falling under Adam, the HIP-graph step equal to the eager step bit for bit.
"""
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import parity_util as PU  # noqa: E402
from parity_util import O  # noqa: E402
from accunet import _lib, kern  # noqa: E402
from accunet import model as M  # noqa: E402
from accunet.loss import WeightedDiceBCE  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def _r(t):
    """t rounded to bf16, as fp64 (the operand the bf16 engine multiplies)."""
    return t.to(BF).double()


def _check_bf16_out(C, ref, K_scale, term_rel=2e-6):
    """C (bf16 or fp32) vs the fp64 reference: bf16 output rounding (2^-8 relative) +
    fp32 accumulation error (term_rel of the sum of |terms|, K_scale)."""
    c = C.double()
    ulp = 2.0 ** -8 if C.dtype == BF else 0.0
    tol = ulp * ref.abs() + term_rel * K_scale + 1e-30
    bad = ((c - ref).abs() > tol)
    assert not bool(bad.any()), (float((c - ref).abs().max()), float(tol.max()))


@pytest.mark.parametrize("M_,N,K", [(4096, 128, 96), (1000, 64, 40), (777, 32, 24),
                                    (2048, 9, 3), (300, 200, 256), (64, 512, 1536),
                                    (65536, 32, 96)])
def test_bf16_row_nt_bias_stats(M_, N, K):
    torch.manual_seed(0)
    A = torch.randn(M_, K, device=DEV).to(BF)
    Wt = torch.randn(N, K, device=DEV)
    b = torch.randn(N, device=DEV)
    C = torch.empty(M_, N, device=DEV, dtype=BF)
    rows = kern.gemm_stats_rows(M_, N, K)
    st = torch.zeros(rows, 2, N, device=DEV, dtype=torch.float64)
    kern.gemm(M_, N, K, a=[A], lda=[K], b=Wt, ldb=K, c=C, ldc=N, bias=b, stats=st)
    ref = A.double() @ _r(Wt).t() + b.double()
    _check_bf16_out(C, ref, (A.double().abs() @ _r(Wt).abs().t()))
    # statistics describe the stored (rounded) C
    cd = C.double()
    s = st.sum(0)
    assert torch.allclose(s[0], cd.sum(0), rtol=1e-9, atol=1e-6)
    assert torch.allclose(s[1], (cd * cd).sum(0), rtol=1e-9, atol=1e-6)


def test_bf16_row_nt_prologue_multisrc_ups():
    torch.manual_seed(1)
    B, H, W = 2, 16, 32
    P = B * H * W
    K1, K2, N = 32, 16, 48
    A1 = torch.randn(P, K1, device=DEV).to(BF)
    base = torch.randn(P, 40, device=DEV).to(BF)
    Wt = torch.randn(N, K1 + K2, device=DEV)
    g2 = torch.randn(B * (H // 2) * (W // 2), N, device=DEV).to(BF)
    g4 = torch.randn(B * (H // 4) * (W // 4), 64, device=DEV).to(BF)
    sc = torch.rand(K1, device=DEV) + 0.5
    sh = torch.randn(K1, device=DEV)
    C = torch.empty(P, N, device=DEV, dtype=BF)
    kern.gemm(P, N, K1 + K2, a=[A1, base], lda=[K1, 40], a_offsets=[0, 8],
              kbeg=[0, K1, K1 + K2], b=Wt, ldb=K1 + K2, c=C, ldc=N, H=H, W=W,
              pro_a=_lib.PRO_AFFINE_LRELU, a_scale=sc, a_shift=sh,
              ups=[(g2, N, 1, 0), (g4, 64, 2, 16)])
    a1 = _r(F.leaky_relu(A1.double() * sc.double() + sh.double(), 0.01))
    X = torch.cat([a1, base[:, 8:24].double()], 1)
    ref = X @ _r(Wt).t()
    up2 = g2.double().view(B, H // 2, W // 2, N).repeat_interleave(2, 1).repeat_interleave(2, 2)
    up4 = g4.double()[:, 16:16 + N].reshape(B, H // 4, W // 4, N).repeat_interleave(4, 1) \
        .repeat_interleave(4, 2)
    ref = ref + up2.reshape(P, N) + up4.reshape(P, N)
    # the activated A is rounded to bf16 from an fp32 (fma) value, the reference from
    # fp64: a few elements round the other way, each worth <= 2^-8 |a| |w|
    _check_bf16_out(C, ref, X.abs() @ _r(Wt).abs().t(), term_rel=2.0 ** -9)


@pytest.mark.parametrize("B,H,W,C,N,k", [(2, 64, 64, 96, 32, 3), (4, 32, 32, 64, 64, 2)])
def test_bf16_dgrad_pyramid_bnb(B, H, W, C, N, k):
    sys.path.insert(0, HERE)
    from test_gemm_gpu import _pyr_bnb_reference
    torch.manual_seed(6)
    P = B * H * W
    J = 2 * k - 1
    dZ = torch.randn(P, N, device=DEV).to(BF)
    Wp = torch.randn(N, J * C, device=DEV) * 0.2
    dP2 = torch.randn(P // 4, 2 * C, device=DEV).to(BF)
    mk2 = torch.randint(0, 4, (P // 4, C), device=DEV, dtype=torch.uint8)
    dP4 = mk4 = None
    if k == 3:
        dP4 = torch.randn(P // 16, 2 * C, device=DEV).to(BF)
        mk4 = torch.randint(0, 16, (P // 16, C), device=DEV, dtype=torch.uint8)
    z = torch.randn(P, C, device=DEV).to(BF)
    st = torch.stack([torch.randn(C), torch.rand(C) + 0.5, torch.rand(C) + 0.5,
                      torch.randn(C) * 0.3]).float().to(DEV)
    R = kern.gemm_stats_rows(P, C, N)
    part = torch.empty(R, 2, C, device=DEV, dtype=torch.float64)
    dA = torch.empty(P, C, device=DEV, dtype=BF)
    kern.gemm(P, C, N, a=[dZ], lda=[N], b=Wp, ldb=J * C, bmode=_lib.BMODE_NN, c=dA, ldc=C,
              H=H, W=W, pyr=(dP2, dP4, mk2, mk4), stats=part, bnb=(z, st, _lib.ACT_LRELU))
    ref, *_ = _pyr_bnb_reference(dZ.double(), _r(Wp), C, B, H, W, dP2.double(),
                                 None if dP4 is None else dP4.double(), mk2, mk4, z.double(), st,
                                 _lib.ACT_LRELU)
    _check_bf16_out(dA, ref, dZ.double().abs() @ _r(Wp)[:, :C].abs() + 4)
    # the BN-backward partials are sums over the stored dA
    pre = z.double() * st[2].double() + st[3].double()
    gg = dA.double() * torch.where(pre > 0, 1.0, 0.01)
    tot = part.sum(0)
    assert torch.allclose(tot[0], gg.sum(0), rtol=1e-6, atol=1e-6 * gg.abs().sum().item())
    assert torch.allclose(tot[1], (gg * (z.double() - st[0].double())).sum(0), rtol=1e-6,
                          atol=1e-6 * gg.abs().sum().item())


@pytest.mark.parametrize("P,Co,Ci,pro", [(65536, 96, 32, 0), (20000, 32, 96, 2),
                                         (4096, 512, 1536, 1), (3000, 9, 3, 0),
                                         (300000, 32, 32, 2)])
def test_bf16_col_nn_wgrad(P, Co, Ci, pro):
    torch.manual_seed(3)
    dZ = torch.randn(P, Co, device=DEV).to(BF)
    X = torch.randn(P, Ci, device=DEV).to(BF)
    sc = torch.rand(Ci, device=DEV) + 0.5
    sh = torch.randn(Ci, device=DEV)
    dW = torch.empty(Co, Ci, device=DEV)
    kern.gemm(Co, Ci, P, a=[dZ], lda=[Co], amode=_lib.AMODE_COL, b=X, ldb=Ci,
              bmode=_lib.BMODE_NN, c=dW, ldc=Ci, pro_b=pro,
              b_scale=sc if pro else None, b_shift=sh if pro else None, allow_split=True)
    Xd = X.double()
    if pro == 1:
        Xd = Xd * sc.double() + sh.double()
    elif pro == 2:
        Xd = F.leaky_relu(Xd * sc.double() + sh.double(), 0.01)
    terms = dZ.double().abs().t() @ Xd.abs()
    if pro:
        # the tiled engine rounds the activated B operand to bf16; the skinny path
        # (small M, N) multiplies it in fp32: either is within one bf16 ulp per term
        Xr = _r(Xd)
        ref_r = dZ.double().t() @ Xr
        ref_f = dZ.double().t() @ Xd
        err = torch.minimum((dW.double() - ref_r).abs(), (dW.double() - ref_f).abs())
        assert bool((err <= 2.0 ** -8 * terms + 1e-6 * terms + 1e-9).all())
    else:
        _check_bf16_out(dW, dZ.double().t() @ Xd, terms)


@pytest.mark.parametrize("B,H,W,Ci,Co", [(2, 32, 32, 32, 32), (1, 16, 64, 64, 64),
                                         (2, 8, 8, 256, 256)])
def test_bf16_conv3x3_fwd_dgrad_wgrad(B, H, W, Ci, Co):
    torch.manual_seed(4)
    x = torch.randn(B, Ci, H, W, dtype=torch.float64).to(BF).double()
    w = torch.randn(Co, Ci, 3, 3, dtype=torch.float64)
    bias = torch.randn(Co, dtype=torch.float64)
    P = B * H * W
    xn = x.permute(0, 2, 3, 1).reshape(P, Ci).to(BF).contiguous().to(DEV)
    wr = w.permute(0, 2, 3, 1).reshape(Co, 9 * Ci).float().contiguous().to(DEV)
    out = torch.empty(P, Co, device=DEV, dtype=BF)
    kern.gemm(P, Co, 9 * Ci, a=[xn], lda=[Ci], amode=_lib.AMODE_SHIFT3, b=wr, ldb=9 * Ci,
              c=out, ldc=Co, bias=bias.float().to(DEV), H=H, W=W, cin=Ci)
    wq = _r(w.float())
    ref = F.conv2d(x, wq, bias.float().double(), padding=1).permute(0, 2, 3, 1).reshape(P, Co)
    terms = F.conv2d(x.abs(), wq.abs(), None, padding=1).permute(0, 2, 3, 1).reshape(P, Co)
    _check_bf16_out(out.cpu(), ref, terms + bias.abs())
    gy = torch.randn(B, Co, H, W, dtype=torch.float64).to(BF).double()
    gyn = gy.permute(0, 2, 3, 1).reshape(P, Co).to(BF).contiguous().to(DEV)
    wf = w.flip(2, 3).permute(1, 2, 3, 0).reshape(Ci, 9 * Co).float().contiguous().to(DEV)
    dx = torch.empty(P, Ci, device=DEV, dtype=BF)
    kern.gemm(P, Ci, 9 * Co, a=[gyn], lda=[Co], amode=_lib.AMODE_SHIFT3, b=wf, ldb=9 * Co,
              c=dx, ldc=Ci, H=H, W=W, cin=Co)
    refx = torch.nn.grad.conv2d_input(x.shape, wq, gy, padding=1).permute(0, 2, 3, 1) \
        .reshape(P, Ci)
    termx = torch.nn.grad.conv2d_input(x.shape, wq.abs(), gy.abs(), padding=1) \
        .permute(0, 2, 3, 1).reshape(P, Ci)
    _check_bf16_out(dx.cpu(), refx, termx)
    dw = torch.empty(Co, 9 * Ci, device=DEV)
    kern.gemm(Co, 9 * Ci, P, a=[gyn], lda=[Co], amode=_lib.AMODE_COL, b=xn, ldb=Ci,
              bmode=_lib.BMODE_NN_SHIFT3, c=dw, ldc=9 * Ci, H=H, W=W, cin=Ci, allow_split=True)
    refw = torch.nn.grad.conv2d_weight(x, w.shape, gy, padding=1).permute(0, 2, 3, 1) \
        .reshape(Co, 9 * Ci)
    termw = torch.nn.grad.conv2d_weight(x.abs(), w.shape, gy.abs(), padding=1) \
        .permute(0, 2, 3, 1).reshape(Co, 9 * Ci)
    _check_bf16_out(dw.cpu(), refw, termw)


# ---------------------------------------------------------------------------
# whole model
#
# Batch-statistic BatchNorm over few values makes small configurations chaotic under
# bf16 perturbation: at n_filts 8 / 4x3x64x64 the emulated-bf16 oracle's gradient is
# ~140 % from fp64 and its outputs ~0.26 (mean) from fp64 logits. Scalars (the loss)
# are then single samples of that noise, so they are compared against the largest
# of an ensemble of emulated runs (inputs jittered below bf16 resolution -> other
# rounding realisations); tensors by their mean and max distance, and the whole
# gradient vector by its relative distance, each within a small factor of the
# emulated run's. The n_filts 32 / 2x3x128x128 case is well conditioned (the
# emulated gradient is a few % from fp64) and checks the same ratios.
# ---------------------------------------------------------------------------
def _oracle_runs(variant, sd, x, mask, training=True, n_jitter=0):
    r64 = PU.oracle_run(variant, sd, x, mask, training=training)
    with O.storage_rounding(BF):
        emu = PU.oracle_run(variant, sd, x, mask, training=training)
        ens = []
        for j in range(n_jitter):
            g = torch.Generator().manual_seed(100 + j)
            xj = x * (1 + (torch.rand(x.shape, generator=g) * 2 - 1) * 2.0 ** -9)
            ens.append(PU.oracle_run(variant, sd, xj, mask, training=training))
    return r64, emu, ens


def _hip_bf16(variant, sd, nf, x, mask, training=True):
    m = M.VARIANTS[variant](3, 1, n_filts=nf, precision="bf16")
    m.load_state_dict(sd)
    m = m.to(DEV).train(training)
    if training:
        out = m(x.to(DEV))
        loss = WeightedDiceBCE(0.5, 0.5)(out, mask.to(DEV))
        loss.backward()
        return m, out.detach(), loss.detach()
    with torch.no_grad():
        return m, m(x.to(DEV)), None


def _compare_bf16_model(variant, nf, B, S, seed, emu_grad_max=None):
    spec = O.param_spec(variant, 3, 1, nf)
    sd = O.det_state_dict(spec, seed=seed)
    x = O.det_input((B, 3, S, S), "golden-x")
    mask = O.det_mask((B, 1, S, S), "golden-mask", p=0.4)
    (o64, l64, g64, sd64), (oe, le, ge, sde), ens = _oracle_runs(variant, sd, x, mask, n_jitter=3)
    m, out, loss = _hip_bf16(variant, sd, nf, x, mask)
    assert out.dtype == torch.float32  # the model output stays fp32
    dh = out.double().cpu() - o64
    de = oe - o64
    assert dh.abs().mean() <= 2 * de.abs().mean() + 1e-7, (float(dh.abs().mean()), float(de.abs().mean()))
    assert dh.abs().max() <= 4 * de.abs().max() + 1e-6, (float(dh.abs().max()), float(de.abs().max()))
    el = max([abs(le.item() - l64.item())] + [abs(r[1].item() - l64.item()) for r in ens])
    assert abs(loss.item() - l64.item()) <= 4 * el + 1e-6, (loss.item(), l64.item(), el)
    keys = [k for k, _ in m.named_parameters()]
    hip = {}
    for k, p in m.named_parameters():
        assert p.grad is None or p.grad.dtype == torch.float32
        hip[k] = p.grad if p.grad is not None else torch.zeros_like(p)
    eg_h = PU.global_rel_err(hip, g64, keys)
    eg_e = max([PU.global_rel_err(ge, g64, keys)] + [PU.global_rel_err(r[2], g64, keys) for r in ens])
    assert eg_h <= 2 * eg_e + 1e-6, (eg_h, eg_e)
    if emu_grad_max is not None:  # the configuration is well conditioned: a meaningful bound
        assert eg_e <= emu_grad_max, eg_e
    msd = m.state_dict()
    bh, be = [], []
    for k, v in sd64.items():
        if k.endswith(("running_mean", "running_var")):
            bh.append((msd[k].double().cpu() - v).abs().mean().item())
            be.append((sde[k].double() - v).abs().mean().item())
        elif k.endswith("num_batches_tracked"):
            assert int(msd[k]) == int(v), k
    assert sum(bh) <= 2 * sum(be) + 1e-9, (sum(bh), sum(be))


@pytest.mark.parametrize("variant", ["canonical", "script", "lite", "w"])
def test_bf16_whole_model_train_step_vs_emulated_oracle(variant):
    _compare_bf16_model(variant, nf=8, B=4, S=64, seed=0)


def test_bf16_full_width_vs_emulated_oracle():
    """canonical n_filts 32 (16.77 M) at 2x3x128x128. Even here the emulated-bf16
    gradient is ~150 % (global relative) from fp64 (the fp32 reference itself is ~5 %
    off at n_filts 8): batch-statistic BatchNorm and the SE gates amplify storage
    rounding, so gradient DIRECTIONS are not a precision bound for this model in bf16;
    the check is that the HIP bf16 run is no noisier than bf16 storage itself."""
    _compare_bf16_model("canonical", nf=32, B=2, S=128, seed=7)


@pytest.mark.parametrize("variant,nf,B,S,seed", [("canonical", 8, 4, 64, 0), ("script", 8, 4, 64, 0),
                                                ("lite", 8, 4, 64, 0), ("w", 8, 4, 64, 0),
                                                ("canonical", 32, 2, 128, 7)])
def test_bf16_eval_mode_gradient_direction(variant, nf, B, S, seed):
    """The gradient-direction bound the batch-statistic runs cannot give: with the
    BatchNorms on their running statistics (model.eval(), the reference's
    ACC_UNet/ACC_UNet.py BatchNorm2d in eval mode) the network is a fixed, well-
    conditioned function, and the emulated-bf16 oracle's gradient is 0.4-0.5 % (global
    relative) from fp64 with cosine 0.99999 (n_filts 8 and 32). The HIP bf16 forward +
    backward (loss WeightedDiceBCE) must stay within 3x the emulated error + 0.2 % of
    the fp64 gradient, point the same way (cosine >= 0.9999), and give the loss within
    3x the emulated loss error."""
    spec = O.param_spec(variant, 3, 1, nf)
    sd = O.det_state_dict(spec, seed=seed)
    x = O.det_input((B, 3, S, S), "golden-x")
    mask = O.det_mask((B, 1, S, S), "golden-mask", p=0.4)
    o64, l64, g64, _ = PU.oracle_run(variant, sd, x, mask, training=False)
    with O.storage_rounding(BF):
        oe, le, ge, _ = PU.oracle_run(variant, sd, x, mask, training=False)
    m = M.VARIANTS[variant](3, 1, n_filts=nf, precision="bf16")
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    out = m(x.to(DEV))
    loss = WeightedDiceBCE(0.5, 0.5)(out, mask.to(DEV))
    loss.backward()
    keys = [k for k, _ in m.named_parameters()]
    hip = {k: (p.grad if p.grad is not None else torch.zeros_like(p)) for k, p in m.named_parameters()}
    eg_e = PU.global_rel_err(ge, g64, keys)
    eg_h = PU.global_rel_err(hip, g64, keys)
    cos = PU.grad_cosine(hip, g64, keys)
    print(f"{variant} nf{nf}: grad rel err hip {eg_h:.3e} emulated {eg_e:.3e}, cos {cos:.7f}")
    assert eg_e < 0.02, eg_e  # the configuration really is well conditioned
    assert eg_h <= 3 * eg_e + 2e-3, (eg_h, eg_e)
    assert cos >= 0.9999, cos
    assert abs(loss.item() - l64.item()) <= 3 * abs(le.item() - l64.item()) + 1e-5
    assert (out.double().cpu() - o64).abs().max() <= 3 * (oe - o64).abs().max() + 1e-5


def test_bf16_training_trajectory_tracks_fp32():
    """What bf16 mixed precision must preserve in practice: 12 Adam steps (lr 1e-3) of
    the canonical model (n_filts 16, 4x3x128x128, fixed batch) from the same weights in
    fp32 and in bf16; the two loss curves stay within 2 % (relative) of each other and
    both fall."""
    from accunet.train import TrainStep
    sd = O.det_state_dict(O.param_spec("canonical", 3, 1, 16), seed=11)
    x = O.det_input((4, 3, 128, 128), "traj16-x").to(DEV)
    mk = O.det_mask((4, 1, 128, 128), "traj16-mask", p=0.3).to(DEV)
    curves = {}
    for prec in ("fp32", "bf16"):
        m = M.VARIANTS["canonical"](3, 1, n_filts=16)
        m.load_state_dict(sd)
        m = m.to(DEV).train()
        step = TrainStep(m, lr=1e-3, precision=prec)
        curves[prec] = [float(step(x, mk)) for _ in range(12)]
    a, b = np.array(curves["fp32"]), np.array(curves["bf16"])
    assert a[-1] < a[0] and b[-1] < b[0], curves
    assert float(np.abs(a - b).max() / a.max()) < 2e-2, curves


def test_bf16_cfg1_lite_shape_eval_and_train():
    """BASELINE configs[0]'s shape (Lite, n_filts 32, 1x3x128x128) in bf16: eval
    probabilities and a train fwd+bwd against the fp64 oracle, 4x the emulated-bf16
    error."""
    spec = O.param_spec("lite", 3, 1, 32)
    sd = O.det_state_dict(spec, seed=1)
    x = O.det_input((1, 3, 128, 128), "cfg1-x")
    mk = O.det_mask((1, 1, 128, 128), "cfg1-mask", p=0.5)
    (o64, _, _, _), (oe, _, _, _), _ = _oracle_runs("lite", sd, x, None, training=False)
    _, pe, _ = _hip_bf16("lite", sd, 32, x, None, training=False)
    e_h = (pe.double().cpu() - o64).abs().max().item()
    e_e = (oe - o64).abs().max().item()
    assert e_h <= 4 * e_e + 1e-5, (e_h, e_e)
    (o64, l64, g64, _), (oe, le, ge, _), _ = _oracle_runs("lite", sd, x, mk)
    m, out, loss = _hip_bf16("lite", sd, 32, x, mk)
    e_h = (out.double().cpu() - o64).abs().max().item()
    e_e = (oe - o64).abs().max().item()
    assert e_h <= 4 * e_e + 1e-5, (e_h, e_e)
    assert abs(loss.item() - l64.item()) <= 4 * abs(le.item() - l64.item()) + 1e-6
    keys = [k for k, _ in m.named_parameters()]
    hip = {k: (p.grad if p.grad is not None else torch.zeros_like(p)) for k, p in m.named_parameters()}
    assert PU.global_rel_err(hip, g64, keys) <= 4 * PU.global_rel_err(ge, g64, keys) + 1e-6


@pytest.mark.parametrize("variant", ["canonical", "lite"])
def test_bf16_hip_graph_step_equals_eager(variant):
    from accunet.train import TrainStep
    nf, B, S = 8, 2, 64
    sd = O.det_state_dict(O.param_spec(variant, 3, 1, nf), seed=0)
    x = O.det_input((B, 3, S, S), "golden-x").to(DEV)
    mask = O.det_mask((B, 1, S, S), "golden-mask", p=0.4).to(DEV)
    runs = {}
    for graph in (False, True):
        m = M.VARIANTS[variant](3, 1, n_filts=nf)
        m.load_state_dict(sd)
        m = m.to(DEV).train()
        step = TrainStep(m, lr=1e-3, graph=graph, precision="bf16")
        losses = [float(step(x, mask).item()) for _ in range(3)]
        runs[graph] = (losses, {k: v.detach().clone() for k, v in m.state_dict().items()})
    assert runs[False][0] == runs[True][0], (runs[False][0], runs[True][0])
    for k, v in runs[False][1].items():
        assert torch.equal(v, runs[True][1][k]), k


def test_bf16_bench_size_properties():
    """BASELINE configs[2] per-GPU shape (canonical, 16x3x256x256) in bf16: two steps
    from one state are bit-identical, probabilities in [0, 1], gradients finite and
    fp32, the loss equals WeightedDiceBCE recomputed in fp64 from the HIP output, the
    initial loss is within 1e-2 of the fp32 mode's, and 4 Adam steps lower the loss."""
    from accunet.train import TrainStep
    torch.manual_seed(0)
    m = M.VARIANTS["canonical"](3, 1, n_filts=32).to(DEV).train()
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(5)
    x = torch.randn(16, 3, 256, 256, generator=g).to(DEV)
    mask = (torch.rand(16, 1, 256, 256, generator=g) < 0.3).float().to(DEV)
    crit = WeightedDiceBCE(0.5, 0.5)
    res = {}
    for prec in ("bf16", "bf16", "fp32"):
        m.set_precision(prec)
        m.load_state_dict(sd0)
        m.zero_grad(set_to_none=True)
        out = m(x)
        loss = crit(out, mask)
        loss.backward()
        res.setdefault(prec, []).append((out.detach().clone(), float(loss.detach()),
                                         [p.grad.detach().clone() for p in m.parameters()
                                          if p.grad is not None]))
    (o1, l1, g1), (o2, l2, g2) = res["bf16"]
    assert torch.equal(o1, o2) and l1 == l2
    assert all(torch.equal(a, b) for a, b in zip(g1, g2))
    assert all(a.dtype == torch.float32 and bool(torch.isfinite(a).all()) for a in g1)
    assert float(o1.min()) >= 0.0 and float(o1.max()) <= 1.0
    ref = O.dice_bce_loss(o1.double().cpu(), mask.double().cpu())
    assert abs(l1 - float(ref)) < 1e-5 * max(1.0, abs(float(ref)))
    l32 = res["fp32"][0][1]
    assert abs(l1 - l32) < 1e-2, (l1, l32)
    m.set_precision("bf16")
    m.load_state_dict(sd0)
    step = TrainStep(m, lr=1e-3, graph=False, precision="bf16")
    losses = [float(step(x, mask)) for _ in range(4)]
    assert losses[-1] < losses[0], losses
