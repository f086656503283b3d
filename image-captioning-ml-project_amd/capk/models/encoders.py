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
from .vit import VIT_ARCHS, CapkViTModel


class ImageEncoder(nn.Module, ABC):
    """Base class for all image encoders (encoders.py:17-34)."""

    @abstractmethod
    def forward(self, images):
        ...


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
        if arch["hidden_size"] != self.feature_dim:
            raise NotImplementedError("capk ViTEncoder: hidden_size != feature_dim projection not on the hot path")
        self.proj = nn.Identity()  # encoders.py:109-113 (hidden == feature_dim)
        if config.freeze:
            for p in self.model.parameters():
                p.requires_grad = False

    def forward(self, images):
        B = images.shape[0]
        seq, pooled = self.model(images)
        N = seq.shape[0] // B
        D = seq.shape[1]
        features = seq.view(B, N, D)[:, 1:]  # encoders.py:122 (drop CLS) — strided view, no copy
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
        if arch["hidden_size"] != self.feature_dim:
            raise NotImplementedError("capk CLIPEncoder: hidden_size != feature_dim projection not on the hot path")
        self.proj = nn.Identity()  # encoders.py:199-203
        if config.freeze:
            for p in self.model.parameters():
                p.requires_grad = False

    def forward(self, images):
        B = images.shape[0]
        seq, pooled = self.model(images)
        N = seq.shape[0] // B
        D = seq.shape[1]
        features = seq.view(B, N, D)[:, 1:]  # encoders.py:213 — strided view of the unnormalised sequence
        mask = torch.ones(B, N - 1, dtype=torch.bool, device=images.device)  # D4 restatement
        return {"features": features, "pooled_features": pooled, "attention_mask": mask}


def build_encoder(config: EncoderConfig) -> ImageEncoder:
    """encoders.py:299-312 (with D2: string types accepted)."""
    et = config.encoder_type if isinstance(config.encoder_type, EncoderType) else EncoderType(config.encoder_type)
    if et == EncoderType.VIT:
        return ViTEncoder(config)
    if et == EncoderType.CLIP:
        return CLIPEncoder(config)
    if et in (EncoderType.RESNET, EncoderType.SWIN):
        raise NotImplementedError(f"capk: encoder '{et.value}' is scheduled after the ViT hot path (SURVEY §8)")
    raise ValueError(f"Unsupported encoder type: {config.encoder_type}")
