"""ResNet image encoder on libcapk kernels.

Module tree and parameter/buffer names mirror transformers 5.15 ``ResNetModel``
(``embedder.embedder.{convolution,normalization}``,
``encoder.stages.{i}.layers.{j}.shortcut.{convolution,normalization}``,
``encoder.stages.{i}.layers.{j}.layer.{0,1,2}.{convolution,normalization}``;
modeling_resnet.py:39-330) so reference checkpoints load unchanged.  The legacy
torchvision trunk of models/encoder.py reuses the same blocks under torchvision
names (``capk.legacy``).

MI355X layout: activations are channels-last rows ``[B*H*W, C]`` (bf16 in the
throughput path), so

  1x1 conv, stride 1     -> one GEMM on the activation rows (no copy)
  KxK / strided conv     -> im2col panel (k order kh, kw, c) + GEMM
  BatchNorm (train mode) -> two-pass column statistics + one fused
                            affine/residual/ReLU pass
  backward               -> dW = dZ^T col, dcol = dZ W, deterministic col2im gather

Conv weights are stored kernel-native in the flat ParamStore: ``[Cout, Kp]`` rows
in (kh, kw, cin) order, zero-padded to Kp = roundup(KH*KW*Cin, 64) for the MFMA
K tiles; ``conv.weight`` is a strided ``[Cout, Cin, KH, KW]`` view of that block,
so state dicts keep PyTorch's layout.
"""
import os

import torch
import torch.nn as nn

from .. import ops
from .common import CapkModule

RESNET_ARCHS = {
    # transformers ResNetConfig fields; weights are random-init offline (no from_pretrained)
    "microsoft/resnet-101": dict(num_channels=3, embedding_size=64, hidden_sizes=(256, 512, 1024, 2048),
                                 depths=(3, 4, 23, 3), downsample_in_first_stage=False,
                                 downsample_in_bottleneck=False),
    "microsoft/resnet-50": dict(num_channels=3, embedding_size=64, hidden_sizes=(256, 512, 1024, 2048),
                                depths=(3, 4, 6, 3), downsample_in_first_stage=False,
                                downsample_in_bottleneck=False),
}

KALIGN = 64  # K granularity of the bf16 GEMM's K-major operands


def _kp(k):
    return (k + KALIGN - 1) // KALIGN * KALIGN


def kernel_layout(conv):
    """Register the kernel-native storage of a bias-free Conv2d weight."""
    Cout, Cin, KH, KW = conv.weight.shape
    K = KH * KW * Cin
    Kp = _kp(K)

    def view(s, Cout=Cout, Cin=Cin, KH=KH, KW=KW, K=K):
        return s[:, :K].view(Cout, KH, KW, Cin).permute(0, 3, 1, 2)

    conv.weight._capk_layout = ((Cout, Kp), view)
    conv._capk_kp = Kp
    return conv


def WK(p, dtype):
    """[Cout, Kp] kernel-layout weight: bf16 shadow or fp32 master."""
    return p._capk_bf16_store if dtype == torch.bfloat16 else p._capk_master_store


def GK(p):
    return p._capk_grad_store


# ------------------------------------------------------------ conv + BN units --
def _direct(conv):
    Cout, Cin, k, _ = conv.weight.shape
    return k == 1 and conv.stride[0] == 1 and conv._capk_kp == Cin


def conv_fwd(conv, x, B, H, W, dt, strides=None):
    """z [B*OH*OW, Cout] = conv(x); returns (z, col, OH, OW)."""
    Cout, Cin, k, _ = conv.weight.shape
    s, pad = conv.stride[0], conv.padding[0]
    OH, OW = ops.conv_out_hw(H, W, k, s, pad)
    if strides is None and _direct(conv):
        col = x
    else:
        col = ops.im2col(x, B, H, W, Cin, k, s, pad, conv._capk_kp, dt, strides=strides)
    z = ops.linear(col, WK(conv.weight, dt))
    return z, col, OH, OW


def conv_bwd(conv, dz, col, B, H, W, dt, *, need_dx=True, dx=None, beta=0.0):
    """dW (kernel layout) = dZ^T col; returns dX [B*H*W, Cin] (written or += beta)."""
    ops.linear_dw(dz, col, GK(conv.weight))
    if not need_dx:
        return None
    Cout, Cin, k, _ = conv.weight.shape
    s, pad = conv.stride[0], conv.padding[0]
    w = WK(conv.weight, dt)
    if _direct(conv):
        if dx is None:
            return ops.linear_dx(dz, w)
        return ops.linear_dx(dz, w, out=dx, beta=beta)
    dcol = ops.linear_dx(dz, w)
    if dx is None:
        dx = torch.empty(B * H * W, Cin, dtype=dz.dtype, device=dz.device)
        beta = 0.0
    ops.col2im(dcol, dx, B, H, W, Cin, k, s, pad, conv._capk_kp, beta)
    return dx


# bottleneck BatchNorms followed directly by their ReLU: backward recomputes the ReLU mask from
# z (already read) instead of re-reading y -- CAPK_BN_OWN_RELU=0 re-reads y (A/B)
_OWN_RELU = os.environ.get("CAPK_BN_OWN_RELU", "1") != "0"


def bn_fwd(bn, z, training, *, residual=None, relu=True):
    """nn.BatchNorm2d (+ residual) (+ ReLU) on channels-last rows; returns (y, mean, rstd)."""
    if training:
        nbt = bn.num_batches_tracked
        if nbt is not None and (nbt.dtype != torch.int64 or not nbt.is_cuda):
            raise TypeError("capk BatchNorm: num_batches_tracked must be an int64 device tensor")
        mean, rstd = ops.bn_stats(z, bn.eps, bn.momentum, bn.running_mean, bn.running_var, nbt)
    else:
        mean, rstd = ops.bn_eval_stats(bn.running_mean, bn.running_var, bn.eps)
    y = ops.bn_apply(z, mean, rstd, bn.weight.detach(), bn.bias.detach(), residual=residual, relu=relu)
    return y, mean, rstd


def bn_bwd(bn, dy, z, mean, rstd, training, *, y_mask=None, own_relu=False, dx=None, dz_out=None):
    """own_relu: the ReLU mask is that of this BatchNorm's own output (no residual in
    between), recomputed from z in the kernels instead of re-reading y."""
    if dx is None:
        dx = torch.empty_like(z)
    ops.bn_bwd(dy, z, mean, rstd, bn.weight.detach(), bn.weight._capk_grad, bn.bias._capk_grad, y_mask=y_mask,
               dx=dx, dz_out=dz_out, batch_stats=training, relu_beta=bn.bias.detach() if own_relu else None)
    return dx


# ----------------------------------------------------------------- modules ----
class ResNetConvLayer(nn.Module):
    """modeling_resnet.py:39-71: Conv2d(bias=False, padding=k//2) + BatchNorm2d (+ ReLU)."""

    def __init__(self, cin, cout, kernel_size=3, stride=1, activation="relu"):
        super().__init__()
        self.convolution = kernel_layout(nn.Conv2d(cin, cout, kernel_size, stride, kernel_size // 2, bias=False))
        self.normalization = nn.BatchNorm2d(cout)
        self.relu = activation is not None


class ResNetShortCut(nn.Module):
    """modeling_resnet.py:95-110: 1x1 Conv2d(stride) + BatchNorm2d."""

    def __init__(self, cin, cout, stride=2):
        super().__init__()
        self.convolution = kernel_layout(nn.Conv2d(cin, cout, 1, stride, bias=False))
        self.normalization = nn.BatchNorm2d(cout)


class BottleneckBlock(CapkModule):
    """Shared launch protocol of the HF and torchvision bottleneck blocks: subclasses
    expose their (conv, bn) pairs through units() / shortcut_units()."""

    def out_hw(self, H, W):
        for c, _ in self.units():
            H, W = ops.conv_out_hw(H, W, c.kernel_size[0], c.stride[0], c.padding[0])
        return H, W

    def forward(self, x, B, H, W):
        OH, OW = self.out_hw(H, W)
        return _BottleneckFn.apply(x, self.units()[0][0].weight, self, B, H, W), OH, OW


class ResNetBottleNeckLayer(BottleneckBlock):
    """modeling_resnet.py:143-190 (v1.5: stride on the 3x3 unless downsample_in_bottleneck)."""

    def __init__(self, cin, cout, stride=1, reduction=4, downsample_in_bottleneck=False):
        super().__init__()
        red = cout // reduction
        self.shortcut = ResNetShortCut(cin, cout, stride) if (cin != cout or stride != 1) else nn.Identity()
        self.layer = nn.Sequential(
            ResNetConvLayer(cin, red, 1, stride if downsample_in_bottleneck else 1),
            ResNetConvLayer(red, red, 3, 1 if downsample_in_bottleneck else stride),
            ResNetConvLayer(red, cout, 1, activation=None),
        )

    def units(self):
        return [(cl.convolution, cl.normalization) for cl in self.layer]

    def shortcut_units(self):
        if isinstance(self.shortcut, nn.Identity):
            return None
        return self.shortcut.convolution, self.shortcut.normalization


class ResNetStage(nn.Module):
    def __init__(self, a, cin, cout, stride, depth):
        super().__init__()
        first = ResNetBottleNeckLayer(cin, cout, stride, downsample_in_bottleneck=a["downsample_in_bottleneck"])
        self.layers = nn.Sequential(first, *[ResNetBottleNeckLayer(cout, cout) for _ in range(depth - 1)])


class _ResNetEncoderStages(nn.Module):
    """modeling_resnet.py:221-259."""

    def __init__(self, a):
        super().__init__()
        hs, ds = a["hidden_sizes"], a["depths"]
        self.stages = nn.ModuleList([ResNetStage(a, a["embedding_size"], hs[0],
                                                 2 if a["downsample_in_first_stage"] else 1, ds[0])])
        for (cin, cout), d in zip(zip(hs, hs[1:]), ds[1:]):
            self.stages.append(ResNetStage(a, cin, cout, 2, d))


def stem_forward(m, images):
    """7x7/2 conv + BN + ReLU + MaxPool2d(3, 2, 1) of module m (m.stem_units() -> (conv, bn))."""
    c = m.stem_units()[0]
    H, W = ops.conv_out_hw(images.shape[2], images.shape[3], c.kernel_size[0], c.stride[0], c.padding[0])
    PH, PW = ops.conv_out_hw(H, W, 3, 2, 1)
    return _StemFn.apply(images, c.weight, m), PH, PW


class _ResNetEmbeddings(CapkModule):
    """modeling_resnet.py:74-92: 7x7/2 conv + BN + ReLU, then MaxPool2d(3, 2, 1)."""

    def __init__(self, a):
        super().__init__()
        self.embedder = ResNetConvLayer(a["num_channels"], a["embedding_size"], 7, 2)

    def stem_units(self):
        return self.embedder.convolution, self.embedder.normalization

    def forward(self, images):
        return stem_forward(self, images)


class CapkResNetModel(CapkModule):
    """ResNetModel (modeling_resnet.py:291-330): embedder -> stages -> AdaptiveAvgPool2d(1).
    forward returns the channels-last last_hidden_state rows [B*h*w, C] and (B, h, w)."""

    def __init__(self, arch):
        super().__init__()
        self.arch = dict(arch)
        self.config = type("ResNetArch", (), dict(arch))()
        self.embedder = _ResNetEmbeddings(arch)
        self.encoder = _ResNetEncoderStages(arch)
        self._init_weights()

    def _init_weights(self):
        # ResNetPreTrainedModel._init_weights: kaiming_normal(fan_out, relu) convs, BN 1/0
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def blocks(self):
        for st in self.encoder.stages:
            for layer in st.layers:
                yield layer

    def forward(self, images):
        B = images.shape[0]
        x, H, W = self.embedder(images)
        for layer in self.blocks():
            x, H, W = layer(x, B, H, W)
        return x, (B, H, W)


# --------------------------------------------------------------- functions --
class _StemFn(torch.autograd.Function):
    """ResNetEmbeddings: images NCHW fp32 -> im2col straight from NCHW -> GEMM -> BN+ReLU
    -> 3x3/2 max-pool (index of the first maximum kept for backward)."""

    @staticmethod
    def forward(ctx, images, anchor, m):
        dt = m.cdtype
        conv, bn = m.stem_units()
        B, C, H, W = images.shape
        images = images.contiguous()
        z, col, OH, OW = conv_fwd(conv, images, B, H, W, dt, strides=(C * H * W, W, 1, H * W))
        y, mean, rstd = bn_fwd(bn, z, m.training, relu=True)
        Cout = z.shape[1]
        p, idx, PH, PW = ops.maxpool_fwd(y, B, OH, OW, Cout, 3, 2, 1)
        ctx.m, ctx.geo = m, (B, OH, OW, Cout)
        ctx.saved = (col, z, y, mean, rstd, idx)
        return p

    @staticmethod
    def backward(ctx, dp):
        m = ctx.m
        dt = m.cdtype
        B, OH, OW, Cout = ctx.geo
        col, z, y, mean, rstd, idx = ctx.saved
        ctx.saved = None
        conv, bn = m.stem_units()
        dy = ops.maxpool_bwd(dp.contiguous(), idx, B, OH, OW, Cout, 3, 2, 1)
        dz = bn_bwd(bn, dy, z, mean, rstd, m.training, y_mask=y, dx=dy)
        ops.linear_dw(dz, col, GK(conv.weight))
        return None, None, None


class _BottleneckFn(torch.autograd.Function):
    """ResNetBottleNeckLayer.forward (modeling_resnet.py:182-190):
    out = relu(bn3(conv3(relu(bn2(conv2(relu(bn1(conv1(x)))))))) + shortcut(x))."""

    @staticmethod
    def forward(ctx, x, anchor, L, B, H, W):
        dt = L.cdtype
        tr = L.training
        (k1, n1), (k2, n2), (k3, n3) = L.units()
        scu = L.shortcut_units()
        z1, col1, H1, W1 = conv_fwd(k1, x, B, H, W, dt)
        y1, mu1, rs1 = bn_fwd(n1, z1, tr)
        z2, col2, H2, W2 = conv_fwd(k2, y1, B, H1, W1, dt)
        y2, mu2, rs2 = bn_fwd(n2, z2, tr)
        z3, _, _, _ = conv_fwd(k3, y2, B, H2, W2, dt)
        if scu is None:
            res, sc = x, None
        else:
            zs, cols, _, _ = conv_fwd(scu[0], x, B, H, W, dt)
            res, mus, rss = bn_fwd(scu[1], zs, tr, relu=False)
            sc = (zs, cols, mus, rss)
        out, mu3, rs3 = bn_fwd(n3, z3, tr, residual=res)
        ctx.L, ctx.geo = L, (B, H, W, H1, W1, H2, W2)
        ctx.saved = (col1, z1, y1, mu1, rs1, col2, z2, y2, mu2, rs2, z3, mu3, rs3, sc, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        L = ctx.L
        dt = L.cdtype
        tr = L.training
        B, H, W, H1, W1, H2, W2 = ctx.geo
        col1, z1, y1, mu1, rs1, col2, z2, y2, mu2, rs2, z3, mu3, rs3, sc, out = ctx.saved
        ctx.saved = None
        (k1, n1), (k2, n2), (k3, n3) = L.units()
        dout = dout.contiguous()
        if sc is None:
            dx = torch.empty_like(dout)  # identity shortcut: dX starts as dout * [out > 0]
            dz3 = bn_bwd(n3, dout, z3, mu3, rs3, tr, y_mask=out, dz_out=dx)
        else:
            ks, ns = L.shortcut_units()
            zs, cols, mus, rss = sc
            dz3 = bn_bwd(n3, dout, z3, mu3, rs3, tr, y_mask=out)
            dzs = bn_bwd(ns, dout, zs, mus, rss, tr, y_mask=out)
            dx = conv_bwd(ks, dzs, cols, B, H, W, dt)
        dy2 = conv_bwd(k3, dz3, y2, B, H2, W2, dt)
        dz2 = bn_bwd(n2, dy2, z2, mu2, rs2, tr, own_relu=_OWN_RELU, y_mask=None if _OWN_RELU else y2, dx=dy2)
        dy1 = conv_bwd(k2, dz2, col2, B, H1, W1, dt)
        dz1 = bn_bwd(n1, dy1, z1, mu1, rs1, tr, own_relu=_OWN_RELU, y_mask=None if _OWN_RELU else y1, dx=dy1)
        conv_bwd(k1, dz1, col1, B, H, W, dt, dx=dx, beta=1.0)
        return dx, None, None, None, None, None


class _ResNetHeadFn(torch.autograd.Function):
    """ResNetEncoder.forward (src/models/encoders.py:60-91) with the SURVEY §0.1 D6
    restatement: features = proj(last_hidden_state.flatten(2).transpose(1, 2)),
    pooled = proj(AdaptiveAvgPool2d(1)(last_hidden_state).flatten(1)).  The channels-last
    rows ARE the flattened/transposed map, so `features` is one GEMM on them.  proj is
    nn.Identity when hidden_sizes[-1] == feature_dim (encoders.py:50-54): features are then
    the map rows themselves and pooled the average-pooled map."""

    @staticmethod
    def forward(ctx, x, anchor, enc, B, H, W):
        ctx.set_materialize_grads(False)
        dt = enc.cdtype
        proj = enc.proj if isinstance(enc.proj, nn.Linear) else None
        C = x.shape[1]
        pooled_raw = ops.avgpool_fwd(x, B, H, W, C, 1, 1)
        ctx.enc, ctx.geo = enc, (B, H, W, C)
        if proj is None:
            ctx.saved = None
            return x.view_as(x), pooled_raw
        wt = proj.weight._capk_bf16 if dt == torch.bfloat16 else proj.weight.detach()
        feats = ops.linear(x, wt, proj.bias.detach())
        pooled = ops.linear(pooled_raw, wt, proj.bias.detach())
        ctx.saved = (x, pooled_raw)
        return feats, pooled

    @staticmethod
    def backward(ctx, dfeat, dpooled):
        enc = ctx.enc
        dt = enc.cdtype
        B, H, W, C = ctx.geo
        proj = enc.proj if isinstance(enc.proj, nn.Linear) else None
        if proj is None:
            dx = dfeat.contiguous() if dfeat is not None else None
            if dpooled is not None:
                dx = ops.avgpool_bwd(dpooled.contiguous(), B, H, W, C, 1, 1,
                                     dx=dx.clone() if dx is not None else None, beta=1.0 if dx is not None else 0.0)
            return dx, None, None, None, None, None
        x, pooled_raw = ctx.saved
        ctx.saved = None
        wt = proj.weight._capk_bf16 if dt == torch.bfloat16 else proj.weight.detach()
        gw, gb = proj.weight._capk_grad, proj.bias._capk_grad
        dx = None
        acc = False
        if dfeat is not None:
            dfeat = dfeat.contiguous()
            ops.linear_dw(dfeat, x, gw)
            ops.colsum(dfeat, gb)
            dx = ops.linear_dx(dfeat, wt)
            acc = True
        if dpooled is not None:
            dpooled = dpooled.contiguous()
            ops.linear_dw(dpooled, pooled_raw, gw, accumulate=acc)
            ops.colsum(dpooled, gb, accumulate=acc)
            dpr = ops.linear_dx(dpooled, wt)
            dx = ops.avgpool_bwd(dpr, B, H, W, C, 1, 1, dx=dx, beta=1.0 if dx is not None else 0.0)
        elif dx is None:
            dx = torch.zeros_like(x)
        return dx, None, None, None, None, None
