"""ORACLE — test infrastructure only, never on the product path.

CPU restatement (plain PyTorch-CPU functional ops, fp32 or fp64) of the ACC-UNet
hot path of prashantkul366/ACC-UNet-Unext, used by tests/, __graft_entry__.smoke()
and bench.py's `cpu_baseline` leg as the CHECKER. The product path
(acc-unet-unext_amd/accunet) never imports this module.

Parity pinning: this restatement is checked against golden vectors produced by
importing the reference modules in the build container
(tests/golden/make_golden.py -> tests/golden/*.npz, test tests/test_oracle_golden.py).

Every function cites the reference file:line whose behaviour it restates
(paths relative to the reference repository root):
  ACC_UNet/ACC_UNet.py        canonical model (inv_fctr 34 at cnv72, Sigmoid head)
  Experiments/nets/ACC_UNet.py  script variant (inv_fctr 3 at cnv72, raw logits)
  ACC_UNet/ACC_UNet_lite.py   Lite (MLFC reduced to its 4 SE layers)
  ACC_UNet/ACC_UNet_w.py      W (learnable MLFC merge weight)
  Experiments/utils.py        WeightedDiceBCE / dice metrics
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

VARIANTS = ("canonical", "script", "lite", "w")
SLOPE = 0.01  # torch.nn.LeakyReLU() default, used at ACC_UNet.py:30,73,170,250,312,416
EPS = 1e-5
MOMENTUM = 0.1

# --------------------------------------------------------------------------
# Parameter specification: names / shapes exactly as the reference state_dict.
# --------------------------------------------------------------------------


def _bn_spec(prefix: str, c: int, out: list):
    # torch.nn.BatchNorm2d(c): weight, bias, running_mean, running_var, num_batches_tracked
    out += [(prefix + ".weight", (c,)), (prefix + ".bias", (c,)),
            (prefix + ".running_mean", (c,)), (prefix + ".running_var", (c,)),
            (prefix + ".num_batches_tracked", ())]


def _conv_spec(prefix, cout, cin, kh, kw, out, groups=1):
    out += [(prefix + ".weight", (cout, cin // groups, kh, kw)), (prefix + ".bias", (cout,))]


def _se_spec(prefix, c, out):
    # ChannelSELayer ACC_UNet/ACC_UNet.py:14-34 (fc1, fc2, bn; r = 8)
    cr = c // 8
    out += [(prefix + ".fc1.weight", (cr, c)), (prefix + ".fc1.bias", (cr,)),
            (prefix + ".fc2.weight", (c, cr)), (prefix + ".fc2.bias", (c,))]
    _bn_spec(prefix + ".bn", c, out)


def _hanc_block_spec(prefix, n_filts, out_ch, k, inv, out):
    # HANCBlock.__init__ ACC_UNet/ACC_UNet.py:229-264 (registration order)
    h = n_filts * inv
    _conv_spec(prefix + ".conv1", h, n_filts, 1, 1, out)
    _bn_spec(prefix + ".norm1", h, out)
    _conv_spec(prefix + ".conv2", h, h, 3, 3, out, groups=h)
    _bn_spec(prefix + ".norm2", h, out)
    _conv_spec(prefix + ".hnc.cnv", n_filts, (2 * k - 1) * h, 1, 1, out)
    _bn_spec(prefix + ".hnc.bn", n_filts, out)
    _bn_spec(prefix + ".norm", n_filts, out)
    _conv_spec(prefix + ".conv3", out_ch, n_filts, 1, 1, out)
    _bn_spec(prefix + ".norm3", out_ch, out)
    _se_spec(prefix + ".sqe", out_ch, out)


def _respath_spec(prefix, c, n_lvl, out):
    # ResPath.__init__ ACC_UNet/ACC_UNet.py:296-320: the (initially empty) ModuleLists
    # convs/bns/sqes are registered before bn/sqe, so their entries come first
    convs, bns, sqes = [], [], []
    for i in range(n_lvl):
        _conv_spec(f"{prefix}.convs.{i}", c, c, 3, 3, convs)
        _bn_spec(f"{prefix}.bns.{i}", c, bns)
        _se_spec(f"{prefix}.sqes.{i}", c, sqes)
    out += convs + bns + sqes
    _bn_spec(prefix + ".bn", c, out)
    _bn_spec(prefix + ".sqe", c, out)


def _cbn_spec(prefix, cin, cout, out):
    # Conv2d_batchnorm ACC_UNet/ACC_UNet.py:151-179
    _conv_spec(prefix + ".conv1", cout, cin, 1, 1, out)
    _bn_spec(prefix + ".batchnorm", cout, out)
    _se_spec(prefix + ".sqe", cout, out)


def _mlfc_spec(prefix, f1, f2, f3, f4, out, weighted=False):
    # MLFC.__init__ ACC_UNet/ACC_UNet.py:338-417 (ModuleList registration order)
    fs = (f1, f2, f3, f4)
    tot = sum(fs)
    if weighted:  # ACC_UNet/ACC_UNet_w.py:354 registers W first
        out.append((prefix + ".W", (1,)))
    groups = {k: [] for k in ("blks", "mrg", "bns", "bns_mrg")}
    # the ModuleLists are registered blks1..4, mrg1..4, bns1..4, bns_mrg1..4 (:363-381)
    for lvl, f in enumerate(fs, 1):
        _cbn_spec(f"{prefix}.cnv_blks{lvl}.0", tot, f, groups["blks"])
    for lvl, f in enumerate(fs, 1):
        _cbn_spec(f"{prefix}.cnv_mrg{lvl}.0", 2 * f, f, groups["mrg"])
    for lvl, f in enumerate(fs, 1):
        _bn_spec(f"{prefix}.bns{lvl}.0", f, groups["bns"])
    for lvl, f in enumerate(fs, 1):
        _bn_spec(f"{prefix}.bns_mrg{lvl}.0", f, groups["bns_mrg"])
    out += groups["blks"] + groups["mrg"] + groups["bns"] + groups["bns_mrg"]
    for lvl, f in enumerate(fs, 1):
        _se_spec(f"{prefix}.sqe{lvl}", f, out)


def cnv72_inv(variant: str) -> int:
    # ACC_UNet/ACC_UNet.py:584 (34) vs Experiments/nets/ACC_UNet.py:584 (3)
    return 3 if variant == "script" else 34


def block_table(variant: str, n_channels: int, n_filts: int):
    """(name, n_filts_in, out_ch, k, inv) for the 18 HANC blocks (ACC_UNet.py:554-592)."""
    f = n_filts
    return [
        ("cnv11", n_channels, f, 3, 3), ("cnv12", f, f, 3, 3),
        ("cnv21", f, 2 * f, 3, 3), ("cnv22", 2 * f, 2 * f, 3, 3),
        ("cnv31", 2 * f, 4 * f, 3, 3), ("cnv32", 4 * f, 4 * f, 3, 3),
        ("cnv41", 4 * f, 8 * f, 2, 3), ("cnv42", 8 * f, 8 * f, 2, 3),
        ("cnv51", 8 * f, 16 * f, 1, 3), ("cnv52", 16 * f, 16 * f, 1, 3),
        ("cnv61", 16 * f, 8 * f, 2, 3), ("cnv62", 8 * f, 8 * f, 2, 3),
        ("cnv71", 8 * f, 4 * f, 3, 3), ("cnv72", 4 * f, 4 * f, 3, cnv72_inv(variant)),
        ("cnv81", 4 * f, 2 * f, 3, 3), ("cnv82", 2 * f, 2 * f, 3, 3),
        ("cnv91", 2 * f, f, 3, 3), ("cnv92", f, f, 3, 3),
    ]


def param_spec(variant: str, n_channels: int = 3, n_classes: int = 1, n_filts: int = 32
               ) -> List[Tuple[str, tuple]]:
    """Ordered state_dict (name, shape) list of the reference model."""
    assert variant in VARIANTS
    f = n_filts
    out: list = []
    blocks = {b[0]: b for b in block_table(variant, n_channels, n_filts)}

    def hb(name):
        _, nf, oc, k, inv = blocks[name]
        _hanc_block_spec(name, nf, oc, k, inv, out)

    # ACC_UNet.__init__ attribute order, ACC_UNet/ACC_UNet.py:549-599
    for n in ("cnv11", "cnv12", "cnv21", "cnv22", "cnv31", "cnv32", "cnv41", "cnv42",
              "cnv51", "cnv52"):
        hb(n)
    for i, (c, nl) in enumerate(((f, 4), (2 * f, 3), (4 * f, 2), (8 * f, 1)), 1):
        _respath_spec(f"rspth{i}", c, nl, out)
    for i in (1, 2, 3):
        _mlfc_spec(f"mlfc{i}", f, 2 * f, 4 * f, 8 * f, out, weighted=(variant == "w"))
    for up, cin, cout, blks in (("up6", 16 * f, 8 * f, ("cnv61", "cnv62")),
                                ("up7", 8 * f, 4 * f, ("cnv71", "cnv72")),
                                ("up8", 4 * f, 2 * f, ("cnv81", "cnv82")),
                                ("up9", 2 * f, f, ("cnv91", "cnv92"))):
        # ConvTranspose2d weight is (in, out, kh, kw)
        out += [(up + ".weight", (cin, cout, 2, 2)), (up + ".bias", (cout,))]
        for b in blks:
            hb(b)
    nout = n_classes if n_classes == 1 else n_classes + 1
    _conv_spec("out", nout, f, 1, 1, out)
    return out


# --------------------------------------------------------------------------
# Deterministic, version-independent parameter / input fill (counter hash).
# --------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def _fnv1a(s: str) -> int:
    h = 0xCBF29CE484222325
    for ch in s.encode():
        h ^= ch
        h = (h * 0x100000001B3) & _M64
    return h


def hash_uniform(key: str, n: int) -> np.ndarray:
    """n values uniform in [-1, 1) from splitmix64(fnv1a(key) + i)."""
    with np.errstate(over="ignore"):
        z = (np.arange(n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
             + np.uint64(_fnv1a(key)))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float64) / float(1 << 24)
    return (2.0 * u - 1.0)


def fan_in(shape) -> int:
    if len(shape) <= 1:
        return 1
    return int(np.prod(shape[1:]))


def det_state_dict(spec, seed: int = 0) -> "OrderedDict[str, torch.Tensor]":
    """Deterministic, version-independent fill of every state_dict entry, in the
    ranges PyTorch's default init uses (U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for conv /
    linear weights and biases); BatchNorm affine and running statistics are
    perturbed away from (1, 0, 0, 1) so parity tests exercise them."""
    names = {n for n, _ in spec}
    shapes = dict(spec)
    sd = OrderedDict()
    for name, shape in spec:
        prefix, leaf = name.rsplit(".", 1)
        n = int(np.prod(shape)) if len(shape) else 1
        if leaf == "num_batches_tracked":
            sd[name] = torch.tensor(0, dtype=torch.long)
            continue
        u = torch.from_numpy(hash_uniform(f"{seed}:{name}", n).reshape(shape))
        if leaf == "running_mean":
            v = 0.1 * u
        elif leaf == "running_var":
            v = 1.0 + 0.5 * u.abs()
        elif prefix + ".running_mean" in names:  # BatchNorm affine
            v = (1.0 + 0.2 * u) if leaf == "weight" else 0.1 * u
        elif leaf == "W":  # ACC_UNet_W merge weight (zeros in the reference init)
            v = 0.3 + 0.2 * u
        elif len(shapes[prefix + ".weight"]) == 1:  # LayerNorm affine (UNeXt)
            v = (1.0 + 0.2 * u) if leaf == "weight" else 0.1 * u
        else:
            wshape = shapes[prefix + ".weight"]
            fi = fan_in(wshape)
            if prefix.startswith("up"):  # ConvTranspose2d (in, out, kh, kw): fan_in = dim 1
                fi = wshape[1] * wshape[2] * wshape[3]
            v = u / math.sqrt(max(fi, 1))
        sd[name] = v.float()
    return sd


def det_input(shape, key="x") -> torch.Tensor:
    n = int(np.prod(shape))
    # approximately N(0,1): sum of 4 uniforms scaled
    u = sum(hash_uniform(f"{key}:{j}", n) for j in range(4)) * math.sqrt(3.0 / 4.0)
    return torch.from_numpy(u.reshape(shape)).float()


def det_mask(shape, key="mask", p=0.5) -> torch.Tensor:
    n = int(np.prod(shape))
    u = 0.5 * (hash_uniform(key, n) + 1.0)
    return torch.from_numpy((u < p).astype(np.float32).reshape(shape))


# --------------------------------------------------------------------------
# Functional forward (NCHW, CPU). State dict entries for running stats are
# updated in place in training mode, exactly like the reference modules.
# --------------------------------------------------------------------------
def lrelu(x):
    return F.leaky_relu(x, SLOPE)


# --------------------------------------------------------------------------
# Storage-rounding emulation (tests of the build's bf16 mode only; the reference
# itself is fp32 throughout). With storage_rounding(torch.bfloat16) active, the
# tensors the build keeps in HBM as bf16 are rounded to bf16 where it stores them,
# and so are their gradients in backward: convolution outputs, GEMM operands (the
# activated input of every dense / 1x1 / transposed convolution and its weights),
# pooled tensors, SE outputs and the residual sums. The depthwise 3x3, the SE gate
# and the head read bf16 activations but compute with fp32 weights and do not round
# their activated inputs. Everything else (BatchNorm / SE statistics, the loss) is
# computed in the oracle's dtype. This measures the error bf16 storage alone causes.
# --------------------------------------------------------------------------
_STORE = None


class _RoundStore(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dt):
        ctx.dt = dt
        return x.to(dt).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dt).to(g.dtype), None


def q(x):
    """x as stored by the build (identity unless storage_rounding is active)."""
    return x if _STORE is None else _RoundStore.apply(x, _STORE)


def qw(w):
    """a GEMM weight operand as the bf16 engine reads it (fp32 master, bf16 operand)."""
    return w if _STORE is None else _RoundStore.apply(w, _STORE)


class storage_rounding:
    """with storage_rounding(torch.bfloat16): forward(...) emulates bf16 storage."""

    def __init__(self, dt):
        self.dt = dt

    def __enter__(self):
        global _STORE
        self.prev, _STORE = _STORE, self.dt
        return self

    def __exit__(self, *exc):
        global _STORE
        _STORE = self.prev


def bn(x, sd, p, training):
    # torch.nn.BatchNorm2d semantics (momentum 0.1, eps 1e-5, unbiased running var)
    if training:
        sd[p + ".num_batches_tracked"] += 1
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"],
                        sd[p + ".weight"], sd[p + ".bias"], training, MOMENTUM, EPS)


def conv(x, sd, p, padding=0, groups=1):
    if groups > 1:  # depthwise (HANCBlock.conv2): fp32 weights / activated input
        return q(F.conv2d(x, sd[p + ".weight"], sd[p + ".bias"], padding=padding, groups=groups))
    return q(F.conv2d(q(x), qw(sd[p + ".weight"]), sd[p + ".bias"], padding=padding))


def se(x, sd, p, training):
    """ChannelSELayer.forward, ACC_UNet/ACC_UNet.py:37-49."""
    b, c = x.shape[:2]
    s = F.adaptive_avg_pool2d(x, 1).view(b, c)
    s = lrelu(F.linear(s, sd[p + ".fc1.weight"], sd[p + ".fc1.bias"]))
    s = torch.sigmoid(F.linear(s, sd[p + ".fc2.weight"], sd[p + ".fc2.bias"]))
    y = x * s.view(b, c, 1, 1)
    return q(lrelu(bn(y, sd, p + ".bn", training)))


def _up(x, f):
    return F.interpolate(x, scale_factor=f, mode="nearest")


def hanc_layer(x, sd, p, k, training):
    """HANCLayer.forward, ACC_UNet/ACC_UNet.py:77-142: neighbourhood pyramid
    concatenated along H then viewed as channels (interleave c*(2k-1)+j)."""
    b, c, h, w = x.shape
    parts = [x]
    if k >= 2:
        parts.append(_up(q(F.avg_pool2d(x, 2)), 2))
    if k >= 3:
        parts.append(_up(q(F.avg_pool2d(x, 4)), 4))
    if k >= 2:
        parts.append(_up(q(F.max_pool2d(x, 2)), 2))
    if k >= 3:
        parts.append(_up(q(F.max_pool2d(x, 4)), 4))
    z = torch.cat(parts, dim=2).view(b, c * (2 * k - 1), h, w)
    return lrelu(bn(conv(z, sd, p + ".cnv"), sd, p + ".bn", training))


def hanc_block(x, sd, p, k, training):
    """HANCBlock.forward, ACC_UNet/ACC_UNet.py:267-286."""
    inp = x
    x = lrelu(bn(conv(x, sd, p + ".conv1"), sd, p + ".norm1", training))
    c = x.shape[1]
    x = lrelu(bn(conv(x, sd, p + ".conv2", padding=1, groups=c), sd, p + ".norm2", training))
    x = hanc_layer(x, sd, p + ".hnc", k, training)
    x = bn(q(x + inp), sd, p + ".norm", training)
    x = lrelu(bn(conv(x, sd, p + ".conv3"), sd, p + ".norm3", training))
    return se(x, sd, p + ".sqe", training)


def respath(x, sd, p, n_lvl, training):
    """ResPath.forward, ACC_UNet/ACC_UNet.py:323-328."""
    for i in range(n_lvl):
        y = lrelu(bn(conv(x, sd, f"{p}.convs.{i}", padding=1), sd, f"{p}.bns.{i}", training))
        x = q(x + se(y, sd, f"{p}.sqes.{i}", training))
    return q(bn(q(lrelu(bn(x, sd, p + ".bn", training))), sd, p + ".sqe", training))


def conv_bn_se(x, sd, p, training):
    """Conv2d_batchnorm.forward, ACC_UNet/ACC_UNet.py:182-186."""
    x = bn(conv(x, sd, p + ".conv1"), sd, p + ".batchnorm", training)
    return se(lrelu(x), sd, p + ".sqe", training)


def mlfc(xs, sd, p, training, variant):
    """MLFC.forward, ACC_UNet/ACC_UNet.py:420-527 (W variant: ACC_UNet_w.py:497-522;
    Lite: ACC_UNet_lite.py:422-429)."""
    x1, x2, x3, x4 = xs
    if variant == "lite":
        return tuple(se(x, sd, f"{p}.sqe{i}", training) for i, x in enumerate(xs, 1))
    down = lambda t: q(F.avg_pool2d(t, 2))
    up = lambda t: _up(t, 2)
    b = x1.shape[0]
    cats = [
        [x1, up(x2), up(up(x3)), up(up(up(x4)))],
        [down(x1), x2, up(x3), up(up(x4))],
        [down(down(x1)), down(x2), x3, up(x4)],
        [down(down(down(x1))), down(down(x2)), down(x3), x4],
    ]
    xc = []
    for lvl in range(4):
        z = conv_bn_se(torch.cat(cats[lvl], dim=1), sd, f"{p}.cnv_blks{lvl + 1}.0", training)
        xc.append(q(lrelu(bn(z, sd, f"{p}.bns{lvl + 1}.0", training))))
    outs = []
    for lvl, xl in enumerate(xs):
        c, h, w = xl.shape[1:]
        merged = torch.cat([xc[lvl], xl], dim=2).view(b, 2 * c, h, w)
        m = conv_bn_se(merged, sd, f"{p}.cnv_mrg{lvl + 1}.0", training)
        if variant == "w":
            wgt = sd[p + ".W"]
            m = q(m * wgt + xl * (1 - wgt))
        else:
            m = q(m + xl)
        outs.append(lrelu(bn(m, sd, f"{p}.bns_mrg{lvl + 1}.0", training)))
    return tuple(se(o, sd, f"{p}.sqe{i}", training) for i, o in enumerate(outs, 1))


def convT(x, sd, p):
    return q(F.conv_transpose2d(q(x), qw(sd[p + ".weight"]), sd[p + ".bias"], stride=2))


def forward(sd, x, variant="canonical", training=True, n_classes=1, return_logits=False):
    """ACC_UNet.forward, ACC_UNet/ACC_UNet.py:601-659 (script variant returns logits,
    Experiments/nets/ACC_UNet.py:654-655). return_logits=True returns the head's pre-sigmoid
    output for every variant (a diagnostic the reference does not expose)."""
    t = training
    x = q(x)
    x2 = hanc_block(hanc_block(x, sd, "cnv11", 3, t), sd, "cnv12", 3, t)
    x3 = hanc_block(hanc_block(F.max_pool2d(x2, 2), sd, "cnv21", 3, t), sd, "cnv22", 3, t)
    x4 = hanc_block(hanc_block(F.max_pool2d(x3, 2), sd, "cnv31", 3, t), sd, "cnv32", 3, t)
    x5 = hanc_block(hanc_block(F.max_pool2d(x4, 2), sd, "cnv41", 2, t), sd, "cnv42", 2, t)
    x6 = hanc_block(hanc_block(F.max_pool2d(x5, 2), sd, "cnv51", 1, t), sd, "cnv52", 1, t)
    x2 = respath(x2, sd, "rspth1", 4, t)
    x3 = respath(x3, sd, "rspth2", 3, t)
    x4 = respath(x4, sd, "rspth3", 2, t)
    x5 = respath(x5, sd, "rspth4", 1, t)
    xs = (x2, x3, x4, x5)
    for i in (1, 2, 3):
        xs = mlfc(xs, sd, f"mlfc{i}", t, variant)
    x2, x3, x4, x5 = xs
    x7 = hanc_block(torch.cat([convT(x6, sd, "up6"), x5], 1), sd, "cnv61", 2, t)
    x7 = hanc_block(x7, sd, "cnv62", 2, t)
    x8 = hanc_block(torch.cat([convT(x7, sd, "up7"), x4], 1), sd, "cnv71", 3, t)
    x8 = hanc_block(x8, sd, "cnv72", 3, t)
    x9 = hanc_block(torch.cat([convT(x8, sd, "up8"), x3], 1), sd, "cnv81", 3, t)
    x9 = hanc_block(x9, sd, "cnv82", 3, t)
    x10 = hanc_block(torch.cat([convT(x9, sd, "up9"), x2], 1), sd, "cnv91", 3, t)
    x10 = hanc_block(x10, sd, "cnv92", 3, t)
    if n_classes == 1:  # the head reads bf16 x10 with fp32 weights, fp32 output
        logits = F.conv2d(x10, sd["out.weight"], sd["out.bias"])
    else:
        logits = conv(x10, sd, "out")
    if variant != "script" and n_classes == 1 and not return_logits:
        return torch.sigmoid(logits)
    return logits


# --------------------------------------------------------------------------
# Loss and metrics, Experiments/utils.py
# --------------------------------------------------------------------------
def weighted_bce(logit, truth, weights=(0.5, 0.5)):
    """WeightedBCE.forward, Experiments/utils.py:28-74 (logits version)."""
    logit = logit.float()
    truth = truth.float().view_as(logit)
    if truth.max() > 1.0:
        truth = (truth > 0).float()
    loss = F.binary_cross_entropy_with_logits(logit, truth, reduction="none")
    pos = (truth > 0.5).float()
    neg = 1.0 - pos
    pw = pos.sum().clamp(min=1.0)
    nw = neg.sum().clamp(min=1.0)
    return (weights[0] * pos * loss / pw + weights[1] * neg * loss / nw).sum()


def weighted_dice(logit, truth, weights=(0.5, 0.5), smooth=1e-5):
    """WeightedDiceLoss.forward, Experiments/utils.py:115-138."""
    b = len(logit)
    p = torch.sigmoid(logit.reshape(b, -1))
    t = truth.reshape(b, -1)
    w = truth.detach().reshape(b, -1) * (weights[1] - weights[0]) + weights[0]
    p = w * p
    t = w * t
    inter = (p * t).sum(-1)
    union = (p * p).sum(-1) + (t * t).sum(-1)
    return (1 - (2 * inter + smooth) / (union + smooth)).mean()


def dice_bce_loss(logit, truth, dice_weight=0.5, bce_weight=0.5):
    """WeightedDiceBCE(0.5, 0.5).forward, Experiments/utils.py:160-171 (train_model.py:719)."""
    return dice_weight * weighted_dice(logit, truth) + bce_weight * weighted_bce(logit, truth)


def show_dice(inputs, targets):
    """WeightedDiceBCE._show_dice, Experiments/utils.py:149-158 (sigmoid applied, then
    sigmoid again inside WeightedDiceLoss; mutates targets)."""
    hard = (torch.sigmoid(inputs) >= 0.5).float()
    targets[targets > 0] = 1
    targets[targets <= 0] = 0
    return 1.0 - weighted_dice(hard, targets)


def dice_on_batch(masks, pred):
    """dice_on_batch, Experiments/utils.py:503-519 (numpy hard Dice, smooth 1e-5)."""
    dices = []
    for i in range(pred.shape[0]):
        p = torch.sigmoid(pred[i][0]).detach().cpu().numpy()
        m = masks[i].detach().cpu().numpy().copy()
        p[p >= 0.5] = 1
        p[p < 0.5] = 0
        m[m > 0] = 1
        m[m <= 0] = 0
        yt, yp = m.flatten(), p.flatten()
        inter = np.sum(yt * yp)
        dices.append((2.0 * inter + 1e-5) / (np.sum(yt) + np.sum(yp) + 1e-5))
    return float(np.mean(dices))


def iou_on_batch(masks, pred):
    """iou_on_batch, Experiments/utils.py:478-494 (jaccard of hard masks)."""
    ious = []
    for i in range(pred.shape[0]):
        p = torch.sigmoid(pred[i][0]).detach().cpu().numpy()
        m = masks[i].detach().cpu().numpy().copy()
        p = (p >= 0.5).astype(np.float64).flatten()
        m = (m > 0).astype(np.float64).flatten()
        inter = np.sum(p * m)
        union = np.sum(np.maximum(p, m))
        ious.append(inter / union if union > 0 else 0.0)
    return float(np.mean(ious))


def cosine_warm_restarts_lr(base_lr, eta_min, T_0, epoch):
    """CosineAnnealingWarmRestarts.get_lr with T_mult=1, Experiments/utils.py:668-784."""
    t_cur = epoch % T_0
    return eta_min + (base_lr - eta_min) * (1 + math.cos(math.pi * t_cur / T_0)) / 2


# --------------------------------------------------------------------------
# Input pipeline: ImageToImage2D.__getitem__, Experiments/Load_Dataset.py:453-487.
# cv2 is absent from this image (and the reference pins no fixture for the resize
# branch): cv2.resize's float rules are restated directly (parity unpinned for
# the resize branch; the no-resize branch is plain numpy/torch arithmetic).
# --------------------------------------------------------------------------
def cv_resize_linear(img: np.ndarray, S: int) -> np.ndarray:
    """cv2.resize(img, (S, S)) default INTER_LINEAR on float data: source coordinate
    (d + 0.5) * in / out - 0.5, clamped at 0; the upper neighbour clamped to the last
    pixel (Load_Dataset.py:465-466)."""
    H, W = img.shape

    def axis(n_in):
        f = (np.arange(S, dtype=np.float64) + 0.5) * (n_in / S) - 0.5
        f = np.maximum(f, 0.0)
        i0 = np.minimum(np.floor(f).astype(np.int64), n_in - 1)
        a = np.where(i0 >= n_in - 1, 0.0, f - i0)
        i1 = np.minimum(i0 + 1, n_in - 1)
        return i0, i1, a

    y0, y1, ay = axis(H)
    x0, x1, ax = axis(W)
    im = img.astype(np.float64)
    top = im[y0][:, x0] * (1 - ax) + im[y0][:, x1] * ax
    bot = im[y1][:, x0] * (1 - ax) + im[y1][:, x1] * ax
    return (top * (1 - ay)[:, None] + bot * ay[:, None]).astype(np.float32)


def cv_resize_nearest(m: np.ndarray, S: int) -> np.ndarray:
    """cv2.resize(..., interpolation=INTER_NEAREST): source index floor(d * in / out)
    (Load_Dataset.py:478-479)."""
    H, W = m.shape
    iy = np.minimum(np.floor(np.arange(S) * (H / S)).astype(np.int64), H - 1)
    ix = np.minimum(np.floor(np.arange(S) * (W / S)).astype(np.int64), W - 1)
    return m[iy][:, ix]


def load_item(img_raw: np.ndarray, mask_raw: np.ndarray, S: int, channel_idx: int = 0):
    """Load_Dataset.py:453-487: channel select, resize if needed, per-image z-score
    (torch mean / unbiased std, + 1e-8), mask resize (nearest) and mask > 0 as int64."""
    img = img_raw[channel_idx]
    if img.shape[0] != S:
        img = cv_resize_linear(img, S)
    t = torch.from_numpy(np.ascontiguousarray(img[None])).float()
    t = (t - t.mean()) / (t.std() + 1e-8)
    m = mask_raw
    if m.shape[0] != S:
        m = cv_resize_nearest(m, S)
    return t, torch.from_numpy((m > 0).astype(np.uint8)).long()


# --------------------------------------------------------------------------
# kernels/dwconv2d (large-kernel depthwise conv, NCHW): depthwise_fwd/launch.cu:12-80
# and the tile fill of depthwise_fwd/kernel.cuh:77-120 (clamped source indices,
# window bounded by pad_h in both directions, zero beyond it). The 3x3 routes of
# the launchers use zero padding (cudnn_convolution / at::conv2d).
# --------------------------------------------------------------------------
def dwconvk(x, w, b, ph, pw, replicate):
    """out[n,c,oh,ow] = b[c] + sum_ij w[c,0,i,j] x[n,c,src(oh-ph+i),src(ow-pw+j)]."""
    N, C, H, W = x.shape
    kh, kw = w.shape[2], w.shape[3]
    oH, oW = H - kh + 1 + 2 * ph, W - kw + 1 + 2 * pw
    if replicate:
        rows = torch.arange(-ph, H + ph)
        cols = torch.arange(-pw, W - 1 + pw + 1)
        xr = x[:, :, rows.clamp(0, H - 1)][:, :, :, cols.clamp(0, W - 1)]
        # kernel.cuh:104: beyond pad_h (rows AND columns) the tile holds 0
        xr = xr * (cols.abs() * 0 + ((cols >= -ph) & (cols <= W - 1 + ph)).to(x.dtype))
    else:
        xr = F.pad(x, (pw, pw, ph, ph))
    out = F.conv2d(xr, w, None, groups=C)
    assert out.shape[2:] == (oH, oW)
    if b is not None:
        out = out + b.view(1, C, 1, 1)
    return out


# --------------------------------------------------------------------------
# UNeXt (Experiments/nets/UNext.py:26-358), NCHW functional restatement. The
# reference module imports timm / torchvision (absent here): parity unpinned by
# reference fixtures; this restatement follows the source line by line.
# --------------------------------------------------------------------------
UNEXT_DIMS = (128, 160, 256)  # embed_dims (:231)


def _ln_spec(prefix, c, out):
    out += [(prefix + ".weight", (c,)), (prefix + ".bias", (c,))]


def _lin_spec(prefix, cout, cin, out):
    out += [(prefix + ".weight", (cout, cin)), (prefix + ".bias", (cout,))]


def _shifted_block_spec(prefix, dim, out):
    # shiftedBlock (:166-201): drop_path (Identity), norm2, mlp = shiftmlp(dim, dim)
    _ln_spec(prefix + ".norm2", dim, out)
    _lin_spec(prefix + ".mlp.fc1", dim, dim, out)          # shiftmlp.fc1 (:46)
    _conv_spec(prefix + ".mlp.dwconv.dwconv", dim, dim, 3, 3, out, groups=dim)  # DWConv :150
    _lin_spec(prefix + ".mlp.fc2", dim, dim, out)          # shiftmlp.fc2 (:50)


def unext_param_spec(n_channels: int = 3, n_classes: int = 1):
    """UNext.__init__ (:231-300) in registration order."""
    d0, d1, d2 = UNEXT_DIMS
    out: list = []
    _conv_spec("encoder1", 16, n_channels, 3, 3, out)
    _conv_spec("encoder2", 32, 16, 3, 3, out)
    _conv_spec("encoder3", d0, 32, 3, 3, out)
    _bn_spec("ebn1", 16, out)
    _bn_spec("ebn2", 32, out)
    _bn_spec("ebn3", d0, out)
    _ln_spec("norm3", d1, out)
    _ln_spec("norm4", d2, out)
    _ln_spec("dnorm3", d1, out)
    _ln_spec("dnorm4", d0, out)
    _shifted_block_spec("block1.0", d1, out)
    _shifted_block_spec("block2.0", d2, out)
    _shifted_block_spec("dblock1.0", d1, out)
    _shifted_block_spec("dblock2.0", d0, out)
    _conv_spec("patch_embed3.proj", d1, d0, 3, 3, out)   # OverlapPatchEmbed :219-221
    _ln_spec("patch_embed3.norm", d1, out)
    _conv_spec("patch_embed4.proj", d2, d1, 3, 3, out)
    _ln_spec("patch_embed4.norm", d2, out)
    _conv_spec("decoder1", d1, d2, 3, 3, out)
    _conv_spec("decoder2", d0, d1, 3, 3, out)
    _conv_spec("decoder3", 32, d0, 3, 3, out)
    _conv_spec("decoder4", 16, 32, 3, 3, out)
    _conv_spec("decoder5", 16, 16, 3, 3, out)
    _bn_spec("dbn1", d1, out)
    _bn_spec("dbn2", d0, out)
    _bn_spec("dbn3", 32, out)
    _bn_spec("dbn4", 16, out)
    _conv_spec("final", n_classes, 16, 1, 1, out)
    return out


def _shift(x, axis, shift_size=5):
    """shiftmlp's pad / chunk / roll / narrow (:86-93, :104-111), NCHW, axis 2 or 3."""
    B, C, H, W = x.shape
    pad = shift_size // 2
    xn = F.pad(x, (pad, pad, pad, pad), "constant", 0)
    xs = torch.chunk(xn, shift_size, 1)
    x_shift = [torch.roll(x_c, sh, axis) for x_c, sh in zip(xs, range(-pad, pad + 1))]
    x_cat = torch.cat(x_shift, 1)
    x_cat = torch.narrow(x_cat, 2, pad, H)
    return torch.narrow(x_cat, 3, pad, W)


def _shiftmlp(x, sd, p, H, W):
    """shiftmlp.forward (:82-118) on tokens (B, N, C)."""
    B, N, C = x.shape
    xn = x.transpose(1, 2).reshape(B, C, H, W)
    xs = _shift(xn, 2).reshape(B, C, H * W).transpose(1, 2)
    x = F.linear(xs, sd[p + ".fc1.weight"], sd[p + ".fc1.bias"])
    Ch = x.shape[-1]
    xd = x.transpose(1, 2).reshape(B, Ch, H, W)
    xd = F.conv2d(xd, sd[p + ".dwconv.dwconv.weight"], sd[p + ".dwconv.dwconv.bias"], padding=1,
                  groups=Ch)
    x = F.gelu(xd.flatten(2).transpose(1, 2))
    xn = x.transpose(1, 2).reshape(B, Ch, H, W)
    xs = _shift(xn, 3).reshape(B, Ch, H * W).transpose(1, 2)
    return F.linear(xs, sd[p + ".fc2.weight"], sd[p + ".fc2.bias"])


def _ln(x, sd, p):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], 1e-5)


def _block(x, sd, p, H, W):
    """shiftedBlock.forward (:198-201): x + mlp(norm2(x))."""
    return x + _shiftmlp(_ln(x, sd, p + ".norm2"), sd, p + ".mlp", H, W)


def _patch_embed(x, sd, p):
    """OverlapPatchEmbed.forward (:223-229): conv 3x3 stride 2 pad 1, flatten, LN."""
    x = F.conv2d(x, sd[p + ".proj.weight"], sd[p + ".proj.bias"], stride=2, padding=1)
    _, _, H, W = x.shape
    return _ln(x.flatten(2).transpose(1, 2), sd, p + ".norm"), H, W


def unext_forward(sd, x, training=True):
    """UNext.forward (:302-358); returns sigmoid probabilities for n_classes == 1."""
    B = x.shape[0]
    cv = lambda t, n: F.conv2d(t, sd[n + ".weight"], sd[n + ".bias"], padding=1)
    up = lambda t: F.interpolate(t, scale_factor=(2, 2), mode="bilinear")
    out = F.relu(F.max_pool2d(bn(cv(x, "encoder1"), sd, "ebn1", training), 2, 2))
    t1 = out
    out = F.relu(F.max_pool2d(bn(cv(out, "encoder2"), sd, "ebn2", training), 2, 2))
    t2 = out
    out = F.relu(F.max_pool2d(bn(cv(out, "encoder3"), sd, "ebn3", training), 2, 2))
    t3 = out
    out, H, W = _patch_embed(out, sd, "patch_embed3")
    out = _block(out, sd, "block1.0", H, W)
    out = _ln(out, sd, "norm3").reshape(B, H, W, -1).permute(0, 3, 1, 2)
    t4 = out
    out, H, W = _patch_embed(out, sd, "patch_embed4")
    out = _block(out, sd, "block2.0", H, W)
    out = _ln(out, sd, "norm4").reshape(B, H, W, -1).permute(0, 3, 1, 2)
    out = F.relu(up(bn(cv(out, "decoder1"), sd, "dbn1", training)))
    out = out + t4
    _, _, H, W = out.shape
    out = _block(out.flatten(2).transpose(1, 2), sd, "dblock1.0", H, W)
    out = _ln(out, sd, "dnorm3").reshape(B, H, W, -1).permute(0, 3, 1, 2)
    out = F.relu(up(bn(cv(out, "decoder2"), sd, "dbn2", training)))
    out = out + t3
    _, _, H, W = out.shape
    out = _block(out.flatten(2).transpose(1, 2), sd, "dblock2.0", H, W)
    out = _ln(out, sd, "dnorm4").reshape(B, H, W, -1).permute(0, 3, 1, 2)
    out = F.relu(up(bn(cv(out, "decoder3"), sd, "dbn3", training)))
    out = out + t2
    out = F.relu(up(bn(cv(out, "decoder4"), sd, "dbn4", training)))
    out = out + t1
    out = F.relu(up(cv(out, "decoder5")))
    out = F.conv2d(out, sd["final.weight"], sd["final.bias"])
    if out.shape[1] == 1:
        out = torch.sigmoid(out)
    return out


def test_image_dice_iou(output, labs):
    """Experiments/test_model.py:30-38,41-48 (batch of 1): pred = output > 0.5,
    dice = 2 sum(l p) / (sum l + sum p + 1e-5), iou = jaccard_score(l, p) (0 when both
    masks are empty: sklearn's zero_division default)."""
    p = (output.detach().cpu().double().numpy().reshape(-1) > 0.5).astype(np.float32)
    lab = labs.detach().cpu().double().numpy().reshape(-1).astype(np.float32)
    dice = 2 * np.sum(lab * p) / (np.sum(lab) + np.sum(p) + 1e-5)
    inter = np.sum((lab > 0) & (p > 0))
    union = np.sum((lab > 0) | (p > 0))
    return float(dice), float(inter / union) if union > 0 else 0.0
