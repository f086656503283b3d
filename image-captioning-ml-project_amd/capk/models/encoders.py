"""Vision-encoder plugin surface — mirrors src/models/encoders.py.

``build_encoder(EncoderConfig) -> ImageEncoder`` and
``ImageEncoder.forward(images) -> {"features", "pooled_features", "attention_mask"}``
keep the reference contract (encoders.py:17-34, 299-312).  Weights are built
from the architecture named by ``pretrained_model_name`` (random init: there is
no network for ``from_pretrained``; load a reference checkpoint with
``load_state_dict`` — the parameter names match).
"""
from abc import ABC, abstractmethod

import torch
import torch.nn as nn

from ..config import EncoderConfig, EncoderType
from .clip import CLIP_ARCHS, CapkCLIPVisionModel
from .. import ops
from .common import CapkModule, G, W, compute_dtype
from .resnet import RESNET_ARCHS, CapkResNetModel, _ResNetHeadFn
from .swin import SWIN_ARCHS, CapkSwinModel, SwinHeadFn
from .vit import VIT_ARCHS, CapkViTModel


class ImageEncoder(nn.Module, ABC):
    """Base class for all image encoders (encoders.py:17-34)."""

    @abstractmethod
    def forward(self, images):
        ...


class _TokenProjFn(torch.autograd.Function):
    """``self.proj`` of the ViT / CLIP encoders when hidden_size != feature_dim
    (encoders.py:108-112, 199-203): features = proj(last_hidden_state[:, 1:]),
    pooled = proj(pooler_output).  The projection runs over every sequence row (the CLS
    row's output is never read: 1 of N rows) so the result keeps the strided-view
    geometry the decoders consume; its backward scatters the patch-row gradient into a
    zero CLS row with one row gather, then dW / db / dX as for any Linear."""

    @staticmethod
    def forward(ctx, seq, pooled, anchor, enc, B, N):
        ctx.set_materialize_grads(False)
        dt = compute_dtype(enc)
        proj = enc.proj
        wt = W(proj.weight, dt)
        out = ops.linear(seq, wt, proj.bias.detach())
        pout = ops.linear(pooled.contiguous(), wt, proj.bias.detach())
        ctx.enc, ctx.B, ctx.N = enc, B, N
        ctx.saved = (seq, pooled)
        F = out.shape[1]
        return out.view(B, N, F)[:, 1:], pout

    @staticmethod
    def backward(ctx, dfeat, dpooled):
        enc, B, N = ctx.enc, ctx.B, ctx.N
        seq, pooled = ctx.saved
        ctx.saved = None
        dt = compute_dtype(enc)
        proj = enc.proj
        wt = W(proj.weight, dt)
        gw, gb = G(proj.weight), G(proj.bias)
        F = proj.weight.shape[0]
        dseq = dpi = None
        acc = False
        if dfeat is not None:
            dfull = ops.zero_(torch.empty(B * N, F, dtype=seq.dtype, device=seq.device))
            idx = torch.arange(N - 1, dtype=torch.int32, device=seq.device)
            ops.gather_rows(dfeat, idx, dfull, B, N - 1, F, dfeat.stride(1), dfeat.stride(0), F, N * F, y_off=F)
            ops.linear_dw(dfull, seq, gw)
            ops.colsum(dfull, gb)
            dseq = ops.linear_dx(dfull, wt)
            acc = True
        if dpooled is not None:
            dpooled = dpooled.contiguous()
            ops.linear_dw(dpooled, pooled.contiguous(), gw, accumulate=acc)
            ops.colsum(dpooled, gb, accumulate=acc)
            dpi = ops.linear_dx(dpooled, wt)
        return dseq, dpi, None, None, None, None


def _token_proj(enc, seq, pooled, B):
    """(features, pooled) of a ViT-style encoder: strided view of the sequence without CLS
    (no copy) when proj is the identity, else _TokenProjFn."""
    N = seq.shape[0] // B
    if isinstance(enc.proj, nn.Linear):
        return _TokenProjFn.apply(seq, pooled, enc.proj.weight, enc, B, N)
    return seq.view(B, N, seq.shape[1])[:, 1:], pooled


class ViTEncoder(ImageEncoder):
    """encoders.py:94-137 on libcapk kernels."""

    def __init__(self, config: EncoderConfig, arch=None):
        super().__init__()
        name = config.pretrained_model_name or "google/vit-base-patch16-224"
        if arch is None:
            if name not in VIT_ARCHS:
                raise ValueError(f"capk ViTEncoder: unknown architecture '{name}' (known: {sorted(VIT_ARCHS)})")
            arch = VIT_ARCHS[name]
        self.model = CapkViTModel(arch)
        self.feature_dim = config.feature_dim
        hidden = arch["hidden_size"]  # encoders.py:108-112
        self.proj = nn.Linear(hidden, self.feature_dim) if hidden != self.feature_dim else nn.Identity()
        if config.freeze:
            for p in self.model.parameters():
                p.requires_grad = False

    def forward(self, images):
        B = images.shape[0]
        seq, pooled = self.model(images)
        N = seq.shape[0] // B
        features, pooled = _token_proj(self, seq, pooled, B)  # encoders.py:122-127 (drop CLS, proj)
        # encoders.py:130-131 returns a float all-ones mask; restated as a bool "valid" mask (D4)
        mask = torch.ones(B, N - 1, dtype=torch.bool, device=images.device)
        return {"features": features, "pooled_features": pooled, "attention_mask": mask}


class CLIPEncoder(ImageEncoder):
    """encoders.py:185-230 on libcapk kernels: features = last_hidden_state[:, 1:]
    (no final LN), pooled = post_layernorm(CLS) (CLIPVisionModel pooler_output)."""

    def __init__(self, config: EncoderConfig, arch=None):
        super().__init__()
        name = config.pretrained_model_name or "openai/clip-vit-base-patch32"  # encoders.py:191-193
        if arch is None:
            if name not in CLIP_ARCHS:
                raise ValueError(f"capk CLIPEncoder: unknown architecture '{name}' (known: {sorted(CLIP_ARCHS)})")
            arch = CLIP_ARCHS[name]
        self.model = CapkCLIPVisionModel(arch)
        self.feature_dim = config.feature_dim
        hidden = arch["hidden_size"]  # encoders.py:199-203
        self.proj = nn.Linear(hidden, self.feature_dim) if hidden != self.feature_dim else nn.Identity()
        if config.freeze:
            for p in self.model.parameters():
                p.requires_grad = False

    def forward(self, images):
        B = images.shape[0]
        seq, pooled = self.model(images)
        N = seq.shape[0] // B
        features, pooled = _token_proj(self, seq, pooled, B)  # encoders.py:213-221 (unnormalised sequence)
        mask = torch.ones(B, N - 1, dtype=torch.bool, device=images.device)  # D4 restatement
        return {"features": features, "pooled_features": pooled, "attention_mask": mask}


class ResNetEncoder(ImageEncoder, CapkModule):
    """encoders.py:37-91 on libcapk kernels.  Restated per SURVEY §0.1 D6:
    the reference applies Linear(2048->768) to the NCHW map (shape error) and returns
    the unprojected pooler output; here features = proj(flattened map) [B, h*w, D] and
    pooled = proj(avg-pooled map) [B, D], mirroring the ViT/CLIP encoders."""

    def __init__(self, config: EncoderConfig, arch=None):
        super().__init__()
        name = config.pretrained_model_name or "microsoft/resnet-50"  # encoders.py:42-44
        if arch is None:
            if name not in RESNET_ARCHS:
                raise ValueError(f"capk ResNetEncoder: unknown architecture '{name}' (known: {sorted(RESNET_ARCHS)})")
            arch = RESNET_ARCHS[name]
        self.model = CapkResNetModel(arch)
        self.feature_dim = config.feature_dim
        hidden = arch["hidden_sizes"][-1]  # encoders.py:50-54
        self.proj = nn.Linear(hidden, self.feature_dim) if hidden != self.feature_dim else nn.Identity()
        if config.freeze:
            for p in self.model.parameters():
                p.requires_grad = False

    def forward(self, images):
        x, (B, H, W) = self.model(images)
        anchor = self.proj.weight if isinstance(self.proj, nn.Linear) else x
        feats, pooled = _ResNetHeadFn.apply(x, anchor, self, B, H, W)
        features = feats.view(B, H * W, feats.shape[1])
        mask = torch.ones(B, H * W, dtype=torch.bool, device=images.device)  # D4 restatement
        return {"features": features, "pooled_features": pooled, "attention_mask": mask}


class SwinEncoder(ImageEncoder):
    """encoders.py:140-182 on libcapk kernels: features = proj(SwinModel
    last_hidden_state) (proj = Linear when hidden_size != feature_dim, encoders.py:153-158),
    pooled = features.mean(dim=1) (encoders.py:172), all-valid mask (D4 restatement)."""

    def __init__(self, config: EncoderConfig, arch=None):
        super().__init__()
        name = config.pretrained_model_name or "microsoft/swin-base-patch4-window7-224"  # encoders.py:145-147
        if arch is None:
            if name not in SWIN_ARCHS:
                raise ValueError(f"capk SwinEncoder: unknown architecture '{name}' (known: {sorted(SWIN_ARCHS)})")
            arch = SWIN_ARCHS[name]
        self.model = CapkSwinModel(arch)
        self.feature_dim = config.feature_dim
        hidden = self.model.num_features
        self.proj = nn.Linear(hidden, self.feature_dim) if hidden != self.feature_dim else nn.Identity()
        if config.freeze:
            for p in self.model.parameters():
                p.requires_grad = False

    def forward(self, images):
        x, (B, H, W) = self.model(images)
        proj = self.proj if isinstance(self.proj, nn.Linear) else None
        feats, pooled = SwinHeadFn.apply(x, self.model.layernorm.weight, self.model, proj, B, H * W)
        features = feats.view(B, H * W, feats.shape[1])
        mask = torch.ones(B, H * W, dtype=torch.bool, device=images.device)  # D4 restatement
        return {"features": features, "pooled_features": pooled, "attention_mask": mask}


def build_encoder(config: EncoderConfig) -> ImageEncoder:
    """encoders.py:299-312 (with D2: string types accepted)."""
    et = config.encoder_type if isinstance(config.encoder_type, EncoderType) else EncoderType(config.encoder_type)
    if et == EncoderType.VIT:
        return ViTEncoder(config)
    if et == EncoderType.CLIP:
        return CLIPEncoder(config)
    if et == EncoderType.RESNET:
        return ResNetEncoder(config)
    if et == EncoderType.SWIN:
        return SwinEncoder(config)
    raise ValueError(f"Unsupported encoder type: {config.encoder_type}")
