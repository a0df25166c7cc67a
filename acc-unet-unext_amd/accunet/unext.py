"""UNeXt (Experiments/nets/UNext.py:26-358) on the MI355X kernels.

Module tree and parameter names follow the reference (state_dict compatible:
encoder1..3, ebn1..3, norm3/norm4/dnorm3/dnorm4, block1/block2/dblock1/dblock2
(shiftedBlock: norm2, mlp.fc1, mlp.dwconv.dwconv, mlp.fc2), patch_embed3/4
(proj, norm), decoder1..5, dbn1..4, final). Activations run NHWC, which is also the
token layout [B, N = H*W, C] of the shifted-MLP stages, so the reference's
transpose / view / flatten round trips between image and token form cost nothing.

Operator mapping (all compute in libaccunet_hip.so):
  Conv2d 3x3 (+bias)           implicit-GEMM conv (ops.conv3x3), BatchNorm statistics
                               in its epilogue; stride 2 (OverlapPatchEmbed.proj :219)
                               = the stride-1 conv + accunet_subsample2
  BatchNorm2d                  finalize + apply (ops.bn_act_add)
  max_pool2d(2) + relu         ops.pool2 + accunet_relu
  LayerNorm                    accunet_layernorm_fwd/bwd
  shiftmlp shifts              accunet_token_shift (H, then W)
  Linear fc1 / fc2             1x1 GEMM (ops.pw_conv)
  DWConv (3x3 depthwise)       ops.dw_conv (the HANC depthwise kernel)
  GELU                         accunet_gelu_fwd/bwd
  relu(interpolate x2) + skip  accunet_up2_relu_add_fwd / accunet_up2_relu_bwd
  final 1x1 + sigmoid          ops.head
Initial weights use PyTorch's default layer init (the reference's timm
trunc_normal_ init, :52-64, is not reproduced: timm is not part of this image);
load a reference state_dict for identical weights.
"""
from __future__ import annotations

import torch
from torch import nn

from . import kern, ops
from ._lib import ACT_NONE


def _empty(shape, like, dtype=torch.float32):
    return torch.empty(shape, dtype=dtype, device=like.device)


# --------------------------------------------------------------------------- ops
class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, eps):
        C = x.shape[-1]
        P = x.numel() // C
        y = torch.empty_like(x)
        mr = _empty((P, 2), x)
        kern.layernorm_fwd(x, g, b, y, mr, P, C, eps)
        ctx.save_for_backward(x, g, mr)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, g, mr = ctx.saved_tensors
        C = x.shape[-1]
        P = x.numel() // C
        dx = torch.empty_like(x)
        dgb = _empty((2 * C,), x)
        part = kern.layernorm_bwd(x, g, mr, dy.contiguous(), dx, dgb, P, C)
        del part
        return dx, dgb[:C].clone(), dgb[C:].clone(), None


def layernorm(x, mod: nn.LayerNorm):
    return _LayerNormFn.apply(x.contiguous(), mod.weight, mod.bias, mod.eps)


class _GeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = torch.empty_like(x)
        kern.gelu_fwd(x, y)
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dx = torch.empty_like(x)
        kern.gelu_bwd(x, dy.contiguous(), dx)
        return dx


def gelu(x):
    return _GeluFn.apply(x.contiguous())


class _ShiftFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, axis):
        B, H, W, C = x.shape
        y = torch.empty_like(x)
        kern.token_shift(x, y, B, H, W, C, axis, 1)
        ctx.axis = axis
        return y

    @staticmethod
    def backward(ctx, dy):
        B, H, W, C = dy.shape
        dx = torch.empty_like(dy)
        kern.token_shift(dy.contiguous(), dx, B, H, W, C, ctx.axis, -1)
        return dx, None


def token_shift(x, axis):
    return _ShiftFn.apply(x.contiguous(), axis)


class _Up2ReluAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, skip):
        B, H, W, C = x.shape
        out = _empty((B, 2 * H, 2 * W, C), x)
        mask = _empty((B, 2 * H, 2 * W, C), x, torch.uint8)
        kern.up2_relu_add_fwd(x, skip, out, mask, B, H, W, C)
        ctx.save_for_backward(mask)
        ctx.dims = (B, H, W, C)
        ctx.has_skip = skip is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        (mask,) = ctx.saved_tensors
        B, H, W, C = ctx.dims
        dout = dout.contiguous()
        dx = _empty((B, H, W, C), dout)
        kern.up2_relu_bwd(dout, mask, dx, B, H, W, C)
        return dx, (dout if ctx.has_skip else None)


def up2_relu_add(x, skip=None):
    return _Up2ReluAddFn.apply(x.contiguous(), skip.contiguous() if skip is not None else None)


class _ReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = torch.empty_like(x)
        kern.relu(x, None, y)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dx = torch.empty_like(y)
        kern.relu(y, dy.contiguous(), dx)
        return dx


def relu(x):
    return _ReluFn.apply(x.contiguous())


class _Subsample2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        B, H, W, C = x.shape
        y = _empty((B, (H + 1) // 2, (W + 1) // 2, C), x)
        kern.subsample2(x, y, B, H, W, C, 0)
        ctx.dims = (B, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        B, H, W, C = ctx.dims
        dx = _empty((B, H, W, C), dy)
        kern.subsample2(dy.contiguous(), dx, B, H, W, C, 1)
        return dx


def subsample2(x):
    return _Subsample2Fn.apply(x)


def conv_bn(x, conv: nn.Conv2d, bn: nn.BatchNorm2d):
    """bn(conv3x3(x)) materialised (the statistics come from the conv's epilogue)."""
    p = ops.conv3x3(x, conv.weight, conv.bias, consumer_bn=bn)
    p.act = ACT_NONE
    return ops.bn_act_add(p, act_after=ACT_NONE).z


# ------------------------------------------------------------------------ modules
class DWConv(nn.Module):
    """UNext.py:150-161 (3x3 depthwise conv with bias)."""

    def __init__(self, dim=768):
        super().__init__()
        self.dwconv = nn.Conv2d(dim, dim, 3, 1, 1, bias=True, groups=dim)


class shiftmlp(nn.Module):  # noqa: N801 (reference name)
    """UNext.py:38-118 (shift_size 5, GELU, no dropout at drop = 0)."""

    def __init__(self, in_features, hidden_features=None, out_features=None, shift_size=5):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.dim = in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.dwconv = DWConv(hidden_features)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.shift_size = shift_size

    def run(self, x):
        """x: [B, H, W, C] tokens -> fc2(shiftW(gelu(dw(fc1(shiftH(x))))))."""
        s = token_shift(x, 0)
        f1 = ops.pw_conv([s], self.fc1.weight, self.fc1.bias).z
        d = ops.dw_conv(f1, self.dwconv.dwconv.weight, self.dwconv.dwconv.bias).z
        s2 = token_shift(gelu(d), 1)
        return ops.pw_conv([s2], self.fc2.weight, self.fc2.bias).z


class shiftedBlock(nn.Module):  # noqa: N801
    """UNext.py:166-201: x + mlp(norm2(x)) (drop_path 0 -> identity)."""

    def __init__(self, dim, mlp_ratio=1.0):
        super().__init__()
        self.drop_path = nn.Identity()
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = shiftmlp(in_features=dim, hidden_features=int(dim * mlp_ratio))

    def run(self, x):
        m = self.mlp.run(layernorm(x, self.norm2))
        return ops.bn_act_add(m, res=x, act_after=ACT_NONE).z


class OverlapPatchEmbed(nn.Module):
    """UNext.py:204-229: conv 3x3 stride 2 pad 1, then LayerNorm over channels."""

    def __init__(self, img_size=224, patch_size=3, stride=2, in_chans=3, embed_dim=768):
        super().__init__()
        if patch_size != 3 or stride != 2:
            raise NotImplementedError("OverlapPatchEmbed: UNext uses patch 3, stride 2")
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=stride,
                              padding=patch_size // 2)
        self.norm = nn.LayerNorm(embed_dim)

    def run(self, x):
        z = ops.conv3x3(x, self.proj.weight, self.proj.bias).z  # stride-1 conv
        return layernorm(subsample2(z), self.norm)


class UNext(nn.Module):
    """UNext.py:231-358 (embed_dims 128/160/256, depths 1/1/1, mlp_ratio 1)."""

    def __init__(self, n_channels=3, n_classes=1, deep_supervision=False, img_size=224,
                 patch_size=16, in_chans=3, embed_dims=(128, 160, 256), **kwargs):
        super().__init__()
        d0, d1, d2 = embed_dims
        self.n_channels, self.n_classes = n_channels, n_classes
        self.encoder1 = nn.Conv2d(n_channels, 16, 3, stride=1, padding=1)
        self.encoder2 = nn.Conv2d(16, 32, 3, stride=1, padding=1)
        self.encoder3 = nn.Conv2d(32, d0, 3, stride=1, padding=1)
        self.ebn1 = nn.BatchNorm2d(16)
        self.ebn2 = nn.BatchNorm2d(32)
        self.ebn3 = nn.BatchNorm2d(d0)
        self.norm3 = nn.LayerNorm(d1)
        self.norm4 = nn.LayerNorm(d2)
        self.dnorm3 = nn.LayerNorm(d1)
        self.dnorm4 = nn.LayerNorm(d0)
        self.block1 = nn.ModuleList([shiftedBlock(d1)])
        self.block2 = nn.ModuleList([shiftedBlock(d2)])
        self.dblock1 = nn.ModuleList([shiftedBlock(d1)])
        self.dblock2 = nn.ModuleList([shiftedBlock(d0)])
        self.patch_embed3 = OverlapPatchEmbed(img_size // 4, 3, 2, d0, d1)
        self.patch_embed4 = OverlapPatchEmbed(img_size // 8, 3, 2, d1, d2)
        self.decoder1 = nn.Conv2d(d2, d1, 3, stride=1, padding=1)
        self.decoder2 = nn.Conv2d(d1, d0, 3, stride=1, padding=1)
        self.decoder3 = nn.Conv2d(d0, 32, 3, stride=1, padding=1)
        self.decoder4 = nn.Conv2d(32, 16, 3, stride=1, padding=1)
        self.decoder5 = nn.Conv2d(16, 16, 3, stride=1, padding=1)
        self.dbn1 = nn.BatchNorm2d(d1)
        self.dbn2 = nn.BatchNorm2d(d0)
        self.dbn3 = nn.BatchNorm2d(32)
        self.dbn4 = nn.BatchNorm2d(16)
        self.final = nn.Conv2d(16, n_classes, kernel_size=1)
        self.soft = nn.Softmax(dim=1)

    def forward(self, x):
        B, C, H, W = x.shape
        if H % 32 or W % 32:
            raise ValueError(f"UNext: H and W must be divisible by 32, got {H}x{W}")
        if C != self.n_channels:
            raise ValueError(f"UNext: expected {self.n_channels} input channels, got {C}")
        x = ops.to_nhwc(x)
        # encoder: relu(maxpool(bn(conv))) (:257-265); relu commutes with the max-pool
        t1 = relu(ops.pool2(conv_bn(x, self.encoder1, self.ebn1)))
        t2 = relu(ops.pool2(conv_bn(t1, self.encoder2, self.ebn2)))
        t3 = relu(ops.pool2(conv_bn(t2, self.encoder3, self.ebn3)))
        # tokenized MLP stages (:268-290)
        out = self.block1[0].run(self.patch_embed3.run(t3))
        t4 = layernorm(out, self.norm3)
        out = self.block2[0].run(self.patch_embed4.run(t4))
        out = layernorm(out, self.norm4)
        # decoder (:293-351): relu(interp(bn(conv))) + skip
        out = up2_relu_add(conv_bn(out, self.decoder1, self.dbn1), t4)
        out = layernorm(self.dblock1[0].run(out), self.dnorm3)
        out = up2_relu_add(conv_bn(out, self.decoder2, self.dbn2), t3)
        out = layernorm(self.dblock2[0].run(out), self.dnorm4)
        out = up2_relu_add(conv_bn(out, self.decoder3, self.dbn3), t2)
        out = up2_relu_add(conv_bn(out, self.decoder4, self.dbn4), t1)
        out = up2_relu_add(ops.conv3x3(out, self.decoder5.weight, self.decoder5.bias).z)
        if self.n_classes == 1:
            y = ops.head(out, self.final.weight, self.final.bias, True)  # sigmoid (:356-357)
        else:
            y = ops.pw_conv([out], self.final.weight, self.final.bias, want_stats=False).z
        return ops.nhwc_to_nchw(y)
