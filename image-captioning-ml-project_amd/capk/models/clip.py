"""CLIP vision encoder on libcapk kernels.

Mirrors transformers 5.15 ``CLIPVisionModel`` (modeling_clip.py:138-177 embeddings,
355-395 encoder layer, 594-656 vision transformer) with identical parameter names
(transformers 5.15 flattens the vision transformer into CLIPVisionModel itself:
``embeddings.{class_embedding,patch_embedding,position_embedding}``, ``pre_layrnorm``,
``encoder.layers.{i}.{self_attn.{k,v,q,out}_proj,layer_norm1,mlp.fc1,mlp.fc2,layer_norm2}``,
``post_layernorm``).

Differences from ViT, all honoured: patch conv without bias; LayerNorm eps 1e-5;
``pre_layrnorm`` on the embeddings; quick_gelu (x*sigmoid(1.702x)) in the MLP; the
sequence output is NOT layer-normed (``features = last_hidden_state[:, 1:]``,
encoders.py:213) and ``pooled = post_layernorm(last_hidden_state[:, 0])``
(modeling_clip.py:650-651).  The encoder layer reuses the pre-LN layer Function of
vit.py through role accessors.
"""
import torch
import torch.nn as nn

from .. import ops
from .._lib import ACT_QUICK_GELU
from ..params import Fused
from .common import G, CapkModule, W, join_dw, mark
from .vit import _ViTLayerFn

CLIP_ARCHS = {
    "openai/clip-vit-base-patch32": dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                                         intermediate_size=3072, image_size=224, patch_size=32, num_channels=3,
                                         layer_norm_eps=1e-5),
    "openai/clip-vit-base-patch16": dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                                         intermediate_size=3072, image_size=224, patch_size=16, num_channels=3,
                                         layer_norm_eps=1e-5),
    "openai/clip-vit-large-patch14": dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                                          intermediate_size=4096, image_size=224, patch_size=14, num_channels=3,
                                          layer_norm_eps=1e-5),
}


class _CLIPEmbeddings(nn.Module):
    def __init__(self, a):
        super().__init__()
        d = a["hidden_size"]
        self.embed_dim = d
        self.class_embedding = nn.Parameter(torch.randn(d))
        self.patch_embedding = nn.Conv2d(a["num_channels"], d, a["patch_size"], a["patch_size"], bias=False)
        self.num_positions = (a["image_size"] // a["patch_size"]) ** 2 + 1
        self.position_embedding = nn.Embedding(self.num_positions, d)


class _CLIPAttention(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.k_proj = nn.Linear(d, d)
        self.v_proj = nn.Linear(d, d)
        self.q_proj = nn.Linear(d, d)
        self.out_proj = nn.Linear(d, d)
        self.qkv_w = Fused([self.q_proj.weight, self.k_proj.weight, self.v_proj.weight])
        self.qkv_b = Fused([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias])

    @property
    def o_proj(self):
        return self.out_proj

    def _capk_fused_groups(self):
        return [self.qkv_w, self.qkv_b]


class _CLIPMLP(nn.Module):
    def __init__(self, d, i):
        super().__init__()
        self.fc1 = nn.Linear(d, i)
        self.fc2 = nn.Linear(i, d)


class CLIPEncoderLayer(CapkModule):
    act = ACT_QUICK_GELU  # CLIPVisionConfig.hidden_act = "quick_gelu"

    def __init__(self, a):
        super().__init__()
        d = a["hidden_size"]
        self.num_heads = a["num_attention_heads"]
        self.eps = a["layer_norm_eps"]
        self.self_attn = _CLIPAttention(d)
        self.layer_norm1 = nn.LayerNorm(d, eps=self.eps)
        self.mlp = _CLIPMLP(d, a["intermediate_size"])
        self.layer_norm2 = nn.LayerNorm(d, eps=self.eps)

    ln1 = property(lambda self: self.layer_norm1)
    ln2 = property(lambda self: self.layer_norm2)
    attn = property(lambda self: self.self_attn)
    fc1 = property(lambda self: self.mlp.fc1)
    fc2 = property(lambda self: self.mlp.fc2)

    def forward(self, x, B, N):
        self.grad_graph = torch.is_grad_enabled()
        return _ViTLayerFn.apply(x, self.self_attn.out_proj.weight, self, B, N)


class _CLIPEncoderStack(nn.Module):
    def __init__(self, a):
        super().__init__()
        self.layers = nn.ModuleList([CLIPEncoderLayer(a) for _ in range(a["num_hidden_layers"])])


class CapkCLIPVisionModel(CapkModule):
    """CLIPVisionModel (modeling_clip.py:594-656)."""

    def __init__(self, arch):
        super().__init__()
        self.arch = dict(arch)
        self.config = type("CLIPVisionArch", (), dict(arch))()
        d = arch["hidden_size"]
        self.embeddings = _CLIPEmbeddings(arch)
        self.pre_layrnorm = nn.LayerNorm(d, eps=arch["layer_norm_eps"])
        self.encoder = _CLIPEncoderStack(arch)
        self.post_layernorm = nn.LayerNorm(d, eps=arch["layer_norm_eps"])
        self._init_weights()

    def _init_weights(self):
        # CLIPPreTrainedModel._init_weights (initializer_factor 1, initializer_range 0.02)
        a = self.arch
        d, nl = a["hidden_size"], a["num_hidden_layers"]
        vm = self
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        e = vm.embeddings
        nn.init.normal_(e.class_embedding, std=d ** -0.5)
        nn.init.normal_(e.patch_embedding.weight, std=0.02)
        nn.init.normal_(e.position_embedding.weight, std=0.02)
        in_std = d ** -0.5 * (2 * nl) ** -0.5
        for L in vm.encoder.layers:
            for lin in (L.self_attn.q_proj, L.self_attn.k_proj, L.self_attn.v_proj):
                nn.init.normal_(lin.weight, std=in_std)
            nn.init.normal_(L.self_attn.out_proj.weight, std=d ** -0.5)
            nn.init.normal_(L.mlp.fc1.weight, std=(2 * d) ** -0.5)
            nn.init.normal_(L.mlp.fc2.weight, std=in_std)

    def _capk_optional_params(self):
        # post_layernorm receives no gradient when the decoder ignores pooled_features
        return [self.post_layernorm.weight, self.post_layernorm.bias]

    def forward(self, images):
        """images [B,C,H,W] -> (last_hidden_state [B*(Np+1), D] flat, pooled [B, D])."""
        a = self.arch
        B = images.shape[0]
        P = a["patch_size"]
        Np = (images.shape[2] // P) * (images.shape[3] // P)
        N = Np + 1
        vm = self
        x = _CLIPEmbedFn.apply(images, vm.embeddings.patch_embedding.weight, self, B, Np)
        for layer in vm.encoder.layers:
            x = layer(x, B, N)
        pooled = _RowLayerNormFn.apply(x, vm.post_layernorm.weight, vm.post_layernorm, B, N)
        return x, pooled


class _CLIPEmbedFn(torch.autograd.Function):
    """CLIPVisionEmbeddings.forward (modeling_clip.py:179-196: bias-free patch conv as
    im2col + GEMM, class embedding, position embedding) + pre_layrnorm (642)."""

    @staticmethod
    def forward(ctx, images, anchor, m, B, Np):
        dt = m.cdtype
        P, D = m.arch["patch_size"], m.arch["hidden_size"]
        e = m.embeddings
        ln = m.pre_layrnorm
        patches = ops.patchify(images, P, dt)
        pe = ops.linear(patches, W(e.patch_embedding.weight, dt).view(D, -1), None)
        x0 = ops.vit_assemble(pe, e.class_embedding.detach(), e.position_embedding.weight.detach(), B, Np, D)
        x, mu, rs = ops.layernorm_fwd(x0, ln.weight.detach(), ln.bias.detach(), ln.eps)
        ctx.m, ctx.B, ctx.Np = m, B, Np
        ctx.saved = (patches, x0, mu, rs)
        return x

    @staticmethod
    def backward(ctx, dx):
        join_dw(dx.device)  # the layers' weight gradients (side stream) are complete from here on
        m, B, Np = ctx.m, ctx.B, ctx.Np
        D = m.arch["hidden_size"]
        patches, x0, mu, rs = ctx.saved
        ctx.saved = None
        e = m.embeddings
        ln = m.pre_layrnorm
        dx0 = ops.layernorm_bwd(dx.contiguous(), x0, ln.weight.detach(), mu, rs, G(ln.weight), G(ln.bias))
        dpatch = ops.vit_assemble_bwd(dx0, B, Np, D, G(e.class_embedding).view(-1),
                                      G(e.position_embedding.weight).view(-1))
        ops.linear_dw(dpatch, patches, G(e.patch_embedding.weight).view(D, -1))
        return None, None, None, None, None


class _RowLayerNormFn(torch.autograd.Function):
    """pooled = LayerNorm(x[:, 0]) over the CLS rows of a [B*N, D] buffer (strided rows,
    no gather): CLIP post_layernorm (modeling_clip.py:650-651)."""

    @staticmethod
    def forward(ctx, x, anchor, ln, B, N):
        D = x.shape[1]
        rows = x.view(B, N, D)[:, 0]
        y, mu, rs = ops.layernorm_fwd(rows, ln.weight.detach(), ln.bias.detach(), ln.eps,
                                      out=torch.empty(B, D, dtype=x.dtype, device=x.device))
        ctx.ln, ctx.B, ctx.N = ln, B, N
        ctx.saved = (x, mu, rs)
        return y

    @staticmethod
    def backward(ctx, dy):
        ln, B, N = ctx.ln, ctx.B, ctx.N
        x, mu, rs = ctx.saved
        ctx.saved = None
        D = x.shape[1]
        dx = torch.zeros_like(x)
        ops.layernorm_bwd(dy.contiguous(), x.view(B, N, D)[:, 0], ln.weight.detach(), mu, rs, G(ln.weight),
                          G(ln.bias), out=dx.view(B, N, D)[:, 0])
        mark(ln.weight)
        mark(ln.bias)
        return dx, None, None, None, None
