"""ACC-UNet drop-in modules (reference ACC_UNet/ACC_UNet.py and its variants).

The module tree — attribute names, registration order and the torch.nn layers
used as parameter containers — is the reference's, so `state_dict()` keys match
(checked against tests/golden/keys_*.json) and `torch.manual_seed(s); ACC_UNet(...)`
draws the same default initialisation. The forward passes are new: activations
stay NHWC in HBM, BatchNorm/LeakyReLU are applied inside the consuming kernels,
HANCLayer / MLFC concatenations are restructured into GEMMs at source resolution,
and every arithmetic op runs in libaccunet_hip.so (see ops.py).

Public classes (same constructor signatures as the reference):
  ACC_UNet(n_channels, n_classes, n_filts=32)         ACC_UNet/ACC_UNet.py:530
  ACC_UNet_Script(n_channels, n_classes, n_filts=32)  Experiments/nets/ACC_UNet.py:530
  ACC_UNet_Lite(n_channels, n_classes, n_filts=32)    ACC_UNet/ACC_UNet_lite.py:432
  ACC_UNet_W(n_channels, n_classes, n_filts=32)       ACC_UNet/ACC_UNet_w.py:534
  and the blocks ChannelSELayer, HANCLayer, Conv2d_batchnorm, Conv2d_channel,
  HANCBlock, ResPath, MLFC (+ MLFC_Lite, MLFC_W).
Block `forward` methods accept NCHW tensors like the reference; the models
chain the blocks' NHWC `run` methods internally.
"""
from __future__ import annotations

import os

import torch
from torch import nn

from . import ops
from ._lib import ACT_LRELU, ACT_NONE
from .ops import Pending


def _nchw_in(x):
    return ops.to_nhwc(x)


def _nchw_out(y):
    if isinstance(y, Pending):
        y = ops.bn_act_add(y).z
    return ops.nhwc_to_nchw(y)


class ChannelSELayer(nn.Module):
    """Squeeze-and-excitation, ACC_UNet/ACC_UNet.py:9-49 (reduction 8)."""

    def __init__(self, num_channels):
        super().__init__()
        self.gp_avg_pool = nn.AdaptiveAvgPool2d(1)
        self.reduction_ratio = 8
        reduced = num_channels // self.reduction_ratio
        self.fc1 = nn.Linear(num_channels, reduced, bias=True)
        self.fc2 = nn.Linear(reduced, num_channels, bias=True)
        self.act = nn.LeakyReLU()
        self.sigmoid = nn.Sigmoid()
        self.bn = nn.BatchNorm2d(num_channels)

    def run(self, x, consumer_bn=None, res=None, res_slot=None):
        """res: return SE(x) + res with the add fused into the SE (see ops.se)."""
        return ops.se(x, self, consumer_bn=consumer_bn, res=res, res_slot=res_slot)

    def forward(self, inp):
        return _nchw_out(self.run(_nchw_in(inp)))


class HANCLayer(nn.Module):
    """Hierarchical aggregation of neighbourhood context, ACC_UNet/ACC_UNet.py:53-142.

    Supports k in {1, 2, 3} (the values ACC-UNet uses)."""

    def __init__(self, in_chnl, out_chnl, k):
        super().__init__()
        if k not in (1, 2, 3):
            raise NotImplementedError("HANCLayer: k in {1, 2, 3} (ACC-UNet uses only these)")
        self.k = k
        self.cnv = nn.Conv2d((2 * k - 1) * in_chnl, out_chnl, kernel_size=(1, 1))
        self.act = nn.LeakyReLU()
        self.bn = nn.BatchNorm2d(out_chnl)

    def run(self, x) -> Pending:
        """x: NHWC tensor or Pending; returns Pending(z, self.bn, LeakyReLU)."""
        return ops.hanc_layer(x, self.cnv.weight, self.cnv.bias, self.k, consumer_bn=self.bn)

    def forward(self, inp):
        return _nchw_out(self.run(_nchw_in(inp)))


class Conv2d_batchnorm(nn.Module):
    """1x1 conv -> BN -> LeakyReLU -> SE, ACC_UNet/ACC_UNet.py:146-186."""

    def __init__(self, num_in_filters, num_out_filters, kernel_size, stride=(1, 1),
                 activation="LeakyReLU"):
        super().__init__()
        self.activation = nn.LeakyReLU()
        self.conv1 = nn.Conv2d(num_in_filters, num_out_filters, kernel_size=kernel_size,
                               stride=stride, padding="same")
        self.batchnorm = nn.BatchNorm2d(num_out_filters)
        self.sqe = ChannelSELayer(num_out_filters)

    def _check(self):
        ks = self.conv1.kernel_size
        if tuple(ks) != (1, 1) or tuple(self.conv1.stride) != (1, 1):
            raise NotImplementedError("Conv2d_batchnorm: only the 1x1 / stride-1 form ACC-UNet uses")

    def run(self, srcs, *, w_off=0, ups=(), weight=None, consumer_bn=None, slots=None,
            wslot=None, res=None, res_slot=None):
        """res: return sqe(...) + res, the add fused into the SE (the MLFC merge)."""
        self._check()
        w = self.conv1.weight if weight is None else weight
        z = ops.pw_conv(srcs, w, self.conv1.bias, w_off=w_off, ups=ups,
                        consumer_bn=self.batchnorm, slots=slots, wslot=wslot)
        return self.sqe.run(z, consumer_bn=consumer_bn, res=res, res_slot=res_slot)

    def forward(self, x):
        return _nchw_out(self.run([_nchw_in(x)]))


class Conv2d_channel(nn.Module):
    """Pointwise conv -> BN -> LeakyReLU -> SE, ACC_UNet/ACC_UNet.py:189-221."""

    def __init__(self, num_in_filters, num_out_filters):
        super().__init__()
        self.activation = nn.LeakyReLU()
        self.conv1 = nn.Conv2d(num_in_filters, num_out_filters, kernel_size=(1, 1), padding="same")
        self.batchnorm = nn.BatchNorm2d(num_out_filters)
        self.sqe = ChannelSELayer(num_out_filters)

    def run(self, srcs):
        z = ops.pw_conv(srcs, self.conv1.weight, self.conv1.bias, consumer_bn=self.batchnorm)
        return self.sqe.run(z)

    def forward(self, x):
        return _nchw_out(self.run([_nchw_in(x)]))


class HANCBlock(nn.Module):
    """Inverted-bottleneck HANC block, ACC_UNet/ACC_UNet.py:224-286."""

    def __init__(self, n_filts, out_channels, k=3, inv_fctr=3):
        super().__init__()
        hidden = n_filts * inv_fctr
        self.conv1 = nn.Conv2d(n_filts, hidden, kernel_size=1)
        self.norm1 = nn.BatchNorm2d(hidden)
        self.conv2 = nn.Conv2d(hidden, hidden, kernel_size=3, padding=1, groups=hidden)
        self.norm2 = nn.BatchNorm2d(hidden)
        self.hnc = HANCLayer(hidden, n_filts, k)
        self.norm = nn.BatchNorm2d(n_filts)
        self.conv3 = nn.Conv2d(n_filts, out_channels, kernel_size=1)
        self.norm3 = nn.BatchNorm2d(out_channels)
        self.sqe = ChannelSELayer(out_channels)
        self.activation = nn.LeakyReLU()

    def run(self, inp: torch.Tensor) -> torch.Tensor:
        """inp: materialised NHWC tensor -> NHWC output of the block's SE."""
        # inp feeds conv1 and the residual add: its two gradient contributions meet in
        # one buffer (the residual's, handed over as it is, is added in conv1's
        # data-gradient epilogue) instead of an autograd elementwise add
        sl = ops.GradSlot()
        z1 = ops.pw_conv([inp], self.conv1.weight, self.conv1.bias, consumer_bn=self.norm1,
                         slots=[sl])
        z2 = ops.dw_conv(z1, self.conv2.weight, self.conv2.bias, consumer_bn=self.norm2)
        z3 = self.hnc.run(z2)
        # x = norm(lrelu(hnc.bn(z3)) + inp)   (ACC_UNet.py:279; no activation after norm)
        r = ops.bn_act_add(z3, res=inp, consumer_bn=self.norm, act_after=ACT_NONE, res_slot=sl)
        z4 = ops.pw_conv([r], self.conv3.weight, self.conv3.bias, consumer_bn=self.norm3)
        return self.sqe.run(z4)

    def forward(self, inp):
        return _nchw_out(self.run(_nchw_in(inp)))


class ResPath(nn.Module):
    """Residual 3x3 skip path, ACC_UNet/ACC_UNet.py:290-328."""

    def __init__(self, in_chnls, n_lvl):
        super().__init__()
        self.convs = nn.ModuleList([])
        self.bns = nn.ModuleList([])
        self.sqes = nn.ModuleList([])
        self.bn = nn.BatchNorm2d(in_chnls)
        self.act = nn.LeakyReLU()
        self.sqe = nn.BatchNorm2d(in_chnls)  # the reference's "sqe" is a BatchNorm2d (:313)
        for _ in range(n_lvl):
            self.convs.append(nn.Conv2d(in_chnls, in_chnls, kernel_size=(3, 3), padding=1))
            self.bns.append(nn.BatchNorm2d(in_chnls))
            self.sqes.append(ChannelSELayer(in_chnls))

    def run(self, x: torch.Tensor, slot=None) -> torch.Tensor:
        """slot: GradSlot for x's gradient (x also feeds the encoder's next pool)."""
        n = len(self.convs)
        for i in range(n):
            # x feeds the 3x3 conv and the residual add: one shared gradient buffer
            sl = slot if (i == 0 and slot is not None) else ops.GradSlot()
            z = ops.conv3x3(x, self.convs[i].weight, self.convs[i].bias, consumer_bn=self.bns[i],
                            slot=sl)
            # x + sqes[i](act(bns[i](z))) (:326): the add fused into the SE's apply pass
            nxt = self.bn if i == n - 1 else None
            x = self.sqes[i].run(z, consumer_bn=nxt, res=x, res_slot=sl)
        if n == 0:
            x = ops.bn_act_add(x, consumer_bn=self.bn, act_after=ACT_LRELU, want_stats=True)
        # sqe(act(bn(x)))
        y = ops.bn_act_add(x, consumer_bn=self.sqe, act_after=ACT_NONE)
        return ops.bn_act_add(y).z

    def forward(self, x):
        return ops.nhwc_to_nchw(self.run(_nchw_in(x)))


_MLFC_PENDING = os.environ.get("ACCUNET_MLFC_PENDING", "1") != "0"


def _log2(f):
    return f.bit_length() - 1


class MLFC(nn.Module):
    """Multi-level feature compilation, ACC_UNet/ACC_UNet.py:332-527."""

    _weighted = False

    def __init__(self, in_filters1, in_filters2, in_filters3, in_filters4, lenn=1):
        super().__init__()
        if self._weighted:
            self.W = nn.Parameter(torch.zeros(1))  # ACC_UNet/ACC_UNet_w.py:354
        self.in_filters1 = in_filters1
        self.in_filters2 = in_filters2
        self.in_filters3 = in_filters3
        self.in_filters4 = in_filters4
        self.in_filters = in_filters1 + in_filters2 + in_filters3 + in_filters4
        self.no_param_up = nn.Upsample(scale_factor=2)
        self.no_param_down = nn.AvgPool2d(2)
        fs = (in_filters1, in_filters2, in_filters3, in_filters4)
        for kind in ("cnv_blks", "cnv_mrg", "bns", "bns_mrg"):
            for lvl in range(1, 5):
                setattr(self, f"{kind}{lvl}", nn.ModuleList([]))
        for _ in range(lenn):
            for lvl, f in enumerate(fs, 1):
                getattr(self, f"cnv_blks{lvl}").append(Conv2d_batchnorm(self.in_filters, f, (1, 1)))
                getattr(self, f"cnv_mrg{lvl}").append(Conv2d_batchnorm(2 * f, f, (1, 1)))
                getattr(self, f"bns{lvl}").append(nn.BatchNorm2d(f))
                getattr(self, f"bns_mrg{lvl}").append(nn.BatchNorm2d(f))
        self.act = nn.LeakyReLU()
        self.sqe1 = ChannelSELayer(in_filters1)
        self.sqe2 = ChannelSELayer(in_filters2)
        self.sqe3 = ChannelSELayer(in_filters3)
        self.sqe4 = ChannelSELayer(in_filters4)

    def _merge(self, mrg, srcs, wm, slots, xl, bn, slot):
        """x_c_l = LReLU(bns_mrg(cnv_mrg(interleave(x_c_l, x_l)) + x_l)) (:489-520): the
        residual add fused into cnv_mrg's SE (the SE output is never written)."""
        return mrg.run(srcs, weight=wm, slots=slots, consumer_bn=bn, res=xl, res_slot=slot)

    def run(self, x1, x2, x3, x4):
        xs = (x1, x2, x3, x4)
        fs = [x.shape[-1] for x in xs]
        offs = [0, fs[0], fs[0] + fs[1], fs[0] + fs[1] + fs[2]]
        # every x_m and every pooled copy has several consumers below: their gradient
        # contributions meet in one GradSlot each instead of autograd's adds
        sl = {(m, l): ops.GradSlot() for m in range(4) for l in range(m, 4)}
        # AvgPool2d(2) chains (:431-485): at[m][l] = x_m resampled down to level l >= m
        at = {(m, m): xs[m] for m in range(4)}
        for m in range(4):
            for l in range(m + 1, 4):
                at[(m, l)] = ops.pool2(at[(m, l - 1)], mode=ops.kern.POOL_AVG, slot=sl[(m, l - 1)])
        finals = [None] * 4
        for i in range(len(self.cnv_blks1)):
            xcs = []
            for l in range(4):
                blk = getattr(self, f"cnv_blks{l + 1}")[i]
                w = blk.conv1.weight
                ws = ops.GradSlot()  # the calls below write disjoint column slices of w
                # levels coarser than l: 1x1 conv at their own resolution, nearest-up add
                ups = []
                for m in range(l + 1, 4):
                    g = ops.pw_conv([xs[m]], w, None, w_off=offs[m], want_stats=False,
                                    slots=[sl[(m, m)]], wslot=ws).z
                    ups.append((g, _log2(1 << (m - l)), 0))
                srcs = [at[(m, l)] for m in range(l + 1)]
                v1 = blk.run(srcs, ups=ups, consumer_bn=getattr(self, f"bns{l + 1}")[i],
                             slots=[sl[(m, l)] for m in range(l + 1)], wslot=ws)
                # act(bns_l(.)) stays pending: the merge conv applies it in its A prologue
                # (and its backward runs bns_l's in the data-gradient epilogue), instead of
                # a materialising pass and its backward (ACCUNET_MLFC_PENDING=0: A/B)
                xcs.append(v1 if _MLFC_PENDING else ops.bn_act_add(v1).z)
            for l in range(4):
                mrg = getattr(self, f"cnv_mrg{l + 1}")[i]
                f = fs[l]
                # interleaved merge channels: 2c = x_c[c], 2c+1 = x_l[c] (:492)
                wm = ops.group_relayout(mrg.conv1.weight.reshape(f, 2 * f), 2, (0, 1))
                finals[l] = self._merge(mrg, [xcs[l], xs[l]], wm, [None, sl[(l, l)]], xs[l],
                                        getattr(self, f"bns_mrg{l + 1}")[i], sl[(l, l)])
        return tuple(getattr(self, f"sqe{l + 1}").run(finals[l]) for l in range(4))

    def forward(self, x1, x2, x3, x4):
        outs = self.run(*[_nchw_in(x) for x in (x1, x2, x3, x4)])
        return tuple(ops.nhwc_to_nchw(o) for o in outs)


class MLFC_W(MLFC):
    """MLFC with the learnable merge weight, ACC_UNet/ACC_UNet_w.py:332-527."""

    _weighted = True

    def _merge(self, mrg, srcs, wm, slots, xl, bn, slot):
        # cnv_mrg(...) * W + x_l * (1 - W) (ACC_UNet_w.py:497-522); x_l's gradient:
        # autograd adds it
        m = mrg.run(srcs, weight=wm, slots=slots)
        return ops.wmerge(m, xl, self.W, consumer_bn=bn)


class MLFC_Lite(MLFC):
    """MLFC bypass (only the four SE layers run), ACC_UNet/ACC_UNet_lite.py:422-429."""

    def run(self, x1, x2, x3, x4):
        return tuple(getattr(self, f"sqe{l + 1}").run(x) for l, x in enumerate((x1, x2, x3, x4)))


class ACC_UNet(nn.Module):
    """ACC-UNet, ACC_UNet/ACC_UNet.py:530-659 (canonical: cnv72 inv_fctr 34, Sigmoid head)."""

    _cnv72_inv = 34
    _sigmoid_head = True
    _mlfc_cls = MLFC

    def __init__(self, n_channels, n_classes, n_filts=32, *, precision="fp32"):
        super().__init__()
        self.n_channels = n_channels
        self.n_classes = n_classes
        self.set_precision(precision)
        f = n_filts
        self.pool = nn.MaxPool2d(2)
        self.cnv11 = HANCBlock(n_channels, f, k=3, inv_fctr=3)
        self.cnv12 = HANCBlock(f, f, k=3, inv_fctr=3)
        self.cnv21 = HANCBlock(f, 2 * f, k=3, inv_fctr=3)
        self.cnv22 = HANCBlock(2 * f, 2 * f, k=3, inv_fctr=3)
        self.cnv31 = HANCBlock(2 * f, 4 * f, k=3, inv_fctr=3)
        self.cnv32 = HANCBlock(4 * f, 4 * f, k=3, inv_fctr=3)
        self.cnv41 = HANCBlock(4 * f, 8 * f, k=2, inv_fctr=3)
        self.cnv42 = HANCBlock(8 * f, 8 * f, k=2, inv_fctr=3)
        self.cnv51 = HANCBlock(8 * f, 16 * f, k=1, inv_fctr=3)
        self.cnv52 = HANCBlock(16 * f, 16 * f, k=1, inv_fctr=3)
        self.rspth1 = ResPath(f, 4)
        self.rspth2 = ResPath(2 * f, 3)
        self.rspth3 = ResPath(4 * f, 2)
        self.rspth4 = ResPath(8 * f, 1)
        M = self._mlfc_cls
        self.mlfc1 = M(f, 2 * f, 4 * f, 8 * f, lenn=1)
        self.mlfc2 = M(f, 2 * f, 4 * f, 8 * f, lenn=1)
        self.mlfc3 = M(f, 2 * f, 4 * f, 8 * f, lenn=1)
        self.up6 = nn.ConvTranspose2d(16 * f, 8 * f, kernel_size=(2, 2), stride=2)
        self.cnv61 = HANCBlock(16 * f, 8 * f, k=2, inv_fctr=3)
        self.cnv62 = HANCBlock(8 * f, 8 * f, k=2, inv_fctr=3)
        self.up7 = nn.ConvTranspose2d(8 * f, 4 * f, kernel_size=(2, 2), stride=2)
        self.cnv71 = HANCBlock(8 * f, 4 * f, k=3, inv_fctr=3)
        self.cnv72 = HANCBlock(4 * f, 4 * f, k=3, inv_fctr=self._cnv72_inv)
        self.up8 = nn.ConvTranspose2d(4 * f, 2 * f, kernel_size=(2, 2), stride=2)
        self.cnv81 = HANCBlock(4 * f, 2 * f, k=3, inv_fctr=3)
        self.cnv82 = HANCBlock(2 * f, 2 * f, k=3, inv_fctr=3)
        self.up9 = nn.ConvTranspose2d(2 * f, f, kernel_size=(2, 2), stride=2)
        self.cnv91 = HANCBlock(2 * f, f, k=3, inv_fctr=3)
        self.cnv92 = HANCBlock(f, f, k=3, inv_fctr=3)
        if n_classes == 1:
            self.out = nn.Conv2d(f, n_classes, kernel_size=(1, 1))
            self.last_activation = nn.Sigmoid() if self._sigmoid_head else None
        else:
            self.out = nn.Conv2d(f, n_classes + 1, kernel_size=(1, 1))
            self.last_activation = None

    def set_precision(self, precision: str):
        """Activation storage of the training / inference step.

        "fp32" (default): the reference's arithmetic (it trains in fp32,
            Experiments/train_model.py:647), fp32 activations and fp32 MFMA GEMMs.
        "bf16": BASELINE configs[2] mixed precision. Activations and activation
            gradients are stored bf16 in HBM and every convolution runs on the bf16
            MFMA engine (v_mfma_f32_32x32x16_bf16, fp32 accumulation); parameters,
            their gradients, the Adam state, the BatchNorm / SE statistics (fp64
            partials, fp32 running stats) and the model output stay fp32.
        Parameters and state_dict are unchanged, so checkpoints move freely between
        the two modes."""
        dt = {"fp32": torch.float32, "bf16": torch.bfloat16}.get(precision)
        if dt is None:
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        self.precision = precision
        self.act_dtype = dt
        return self

    # pyramid level (resolution H >> level) of every HANCBlock (ACC_UNet.py:605-651)
    _BLOCK_LEVEL = {"cnv11": 0, "cnv12": 0, "cnv21": 1, "cnv22": 1, "cnv31": 2, "cnv32": 2,
                    "cnv41": 3, "cnv42": 3, "cnv51": 4, "cnv52": 4, "cnv61": 3, "cnv62": 3,
                    "cnv71": 2, "cnv72": 2, "cnv81": 1, "cnv82": 1, "cnv91": 0, "cnv92": 0}
    # the depthwise kernels address one image of a block's hidden tensor through a 32-bit
    # buffer descriptor (csrc/dwconv.hip: dw_image_ok)
    DW_IMAGE_LIMIT = 1 << 31

    def check_input_size(self, H, W):
        """Raise ValueError for a spatial size this build cannot run: H, W not divisible
        by 16 (the reference fails there too, in its pooling / cat), or a HANCBlock whose
        depthwise input would reach 2 GiB per image (e.g. canonical cnv72's 4352 hidden
        channels at (H/4)^2 = 352^2 fp32, an input of 1408^2; the reference accepts it)."""
        if H % 16 or W % 16:
            raise ValueError(f"ACC_UNet: H and W must be divisible by 16, got {H}x{W}")
        elem = torch.finfo(self.act_dtype).bits // 8
        for name, lvl in self._BLOCK_LEVEL.items():
            hidden = getattr(self, name).conv2.weight.shape[0]
            nbytes = (H >> lvl) * (W >> lvl) * hidden * elem
            if nbytes >= self.DW_IMAGE_LIMIT:
                raise ValueError(
                    f"ACC_UNet: {name}'s depthwise input is {nbytes / 2**30:.2f} GiB per image "
                    f"at {H}x{W} ({hidden} channels at {H >> lvl}x{W >> lvl}, "
                    f"{self.precision}); the depthwise kernels address one image with 32-bit "
                    f"offsets, limit 2 GiB per image")

    def forward(self, x):
        B, C, H, W = x.shape
        self.check_input_size(H, W)
        if C != self.n_channels:
            raise ValueError(f"ACC_UNet: expected {self.n_channels} input channels, got {C}")
        x1 = ops.to_nhwc(x, self.act_dtype)
        # each encoder output feeds the next level's pool and its ResPath: one shared
        # gradient buffer per level (see ops.GradSlot)
        s2, s3, s4, s5 = (ops.GradSlot() for _ in range(4))
        x2 = self.cnv12.run(self.cnv11.run(x1))
        x3 = self.cnv22.run(self.cnv21.run(ops.pool2(x2, slot=s2)))
        x4 = self.cnv32.run(self.cnv31.run(ops.pool2(x3, slot=s3)))
        x5 = self.cnv42.run(self.cnv41.run(ops.pool2(x4, slot=s4)))
        x6 = self.cnv52.run(self.cnv51.run(ops.pool2(x5, slot=s5)))
        x2 = self.rspth1.run(x2, s2)
        x3 = self.rspth2.run(x3, s3)
        x4 = self.rspth3.run(x4, s4)
        x5 = self.rspth4.run(x5, s5)
        x2, x3, x4, x5 = self.mlfc1.run(x2, x3, x4, x5)
        x2, x3, x4, x5 = self.mlfc2.run(x2, x3, x4, x5)
        x2, x3, x4, x5 = self.mlfc3.run(x2, x3, x4, x5)
        # torch.cat([up(x), skip], dim=1): the ConvT output shuffled straight into the
        # concatenated tensor (ops.conv_transpose2x2_cat)
        upcat = lambda m, t, skip: ops.conv_transpose2x2_cat(t, m.weight, m.bias, skip)
        x7 = self.cnv62.run(self.cnv61.run(upcat(self.up6, x6, x5)))
        x8 = self.cnv72.run(self.cnv71.run(upcat(self.up7, x7, x4)))
        x9 = self.cnv82.run(self.cnv81.run(upcat(self.up8, x8, x3)))
        x10 = self.cnv92.run(self.cnv91.run(upcat(self.up9, x9, x2)))
        if self.out.weight.shape[0] == 1:
            y = ops.head(x10, self.out.weight, self.out.bias, self.last_activation is not None)
        else:
            y = ops.pw_conv([x10], self.out.weight, self.out.bias, want_stats=False).z
        return ops.nhwc_to_nchw(y)


class ACC_UNet_Script(ACC_UNet):
    """The variant Experiments/train_model.py trains (Experiments/nets/ACC_UNet.py:530-662):
    cnv72 inv_fctr 3 and raw logits (no Sigmoid)."""

    _cnv72_inv = 3
    _sigmoid_head = False


class ACC_UNet_Lite(ACC_UNet):
    """ACC_UNet/ACC_UNet_lite.py:432-561 (MLFC bypassed)."""

    _mlfc_cls = MLFC_Lite


class ACC_UNet_W(ACC_UNet):
    """ACC_UNet/ACC_UNet_w.py:534-663 (learnable MLFC merge weight)."""

    _mlfc_cls = MLFC_W


VARIANTS = {"canonical": ACC_UNet, "script": ACC_UNet_Script, "lite": ACC_UNet_Lite,
            "w": ACC_UNet_W}
