"""ViT / ViT-B-16 image encoder on libcapk kernels.

Module tree and parameter names mirror transformers 5.15 ``ViTModel``
(``embeddings.cls_token``, ``embeddings.position_embeddings``,
``embeddings.patch_embeddings.projection``, ``layers.{i}.attention.{q,k,v,o}_proj``,
``layers.{i}.layernorm_before/after``, ``layers.{i}.mlp.fc1/fc2``, ``layernorm``,
``pooler.dense``) so reference checkpoints load unchanged.  The arithmetic is
re-expressed as launches of hand-written gfx950 kernels:

  patchify (im2col, HBM-bound) -> patch GEMM (MFMA) -> CLS/pos assembly
  per layer: LN -> fused QKV GEMM (+bias) -> fused attention -> O GEMM (+bias+residual)
             -> LN -> FC1 GEMM (+bias+GELU, pre-activation kept) -> FC2 GEMM (+bias+residual)
  final LN -> pooler GEMM (+bias+tanh) on the CLS rows

Activations live as [B*(N+1), D] row-major buffers; heads are addressed by
stride, so there are no transposes anywhere.
"""
import math
import os

import torch
import torch.nn as nn

from .. import ops
from .._lib import ACT_DERIV, ACT_GELU_ERF, ACT_TANH
from ..params import Fused, notify_final, store_of
from .common import G, CapkModule, W, heads, join_dw, linear_bwd, mark

# CAPK_ATTN_BIAS=1: the QKV bias gradient from the attention backward (capk_attention_bwd_bias;
# on the ViT shape the fused single-pass kernel sums the dQ / dK / dV it stores per (image, head),
# round 6).  Default off: measured as a loss twice -- round 4 on the split kernels (5240 -> 5122
# img/s, their dQ kernel spilled), round 6 on the fused kernel (5599 -> 5546 img/s same box ABAB,
# profiles/round6/attn_bias_ab.txt: the per-workgroup reduction tail runs at one workgroup per
# CU, 12 rounds a layer, and costs more than the 232 MB column-sum pass it replaces).
_ATTN_BIAS = os.environ.get("CAPK_ATTN_BIAS", "0") == "1"

VIT_ARCHS = {
    # pretrained_model_name -> architecture (weights are random-init offline or loaded from a checkpoint)
    "google/vit-base-patch16-224": dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                                        intermediate_size=3072, image_size=224, patch_size=16, num_channels=3,
                                        layer_norm_eps=1e-12),
    "google/vit-base-patch16-224-in21k": dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                                              intermediate_size=3072, image_size=224, patch_size=16,
                                              num_channels=3, layer_norm_eps=1e-12),
    "google/vit-large-patch16-224": dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                                         intermediate_size=4096, image_size=224, patch_size=16, num_channels=3,
                                         layer_norm_eps=1e-12),
}


def _trunc(t, std=0.02):
    nn.init.trunc_normal_(t, mean=0.0, std=std)


class _PatchEmbeddings(nn.Module):
    def __init__(self, a):
        super().__init__()
        self.projection = nn.Conv2d(a["num_channels"], a["hidden_size"], a["patch_size"], a["patch_size"])


class _Embeddings(nn.Module):
    def __init__(self, a):
        super().__init__()
        n = (a["image_size"] // a["patch_size"]) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, a["hidden_size"]))
        self.position_embeddings = nn.Parameter(torch.zeros(1, n + 1, a["hidden_size"]))
        self.patch_embeddings = _PatchEmbeddings(a)


class _Attention(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.q_proj = nn.Linear(d, d)
        self.k_proj = nn.Linear(d, d)
        self.v_proj = nn.Linear(d, d)
        self.o_proj = nn.Linear(d, d)
        self.qkv_w = Fused([self.q_proj.weight, self.k_proj.weight, self.v_proj.weight])
        self.qkv_b = Fused([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias])

    def _capk_fused_groups(self):
        return [self.qkv_w, self.qkv_b]


class _MLP(nn.Module):
    def __init__(self, d, i):
        super().__init__()
        self.fc1 = nn.Linear(d, i)
        self.fc2 = nn.Linear(i, d)


class ViTLayer(CapkModule):
    def __init__(self, a):
        super().__init__()
        d = a["hidden_size"]
        self.num_heads = a["num_attention_heads"]
        self.eps = a["layer_norm_eps"]
        self.attention = _Attention(d)
        self.layernorm_before = nn.LayerNorm(d, eps=self.eps)
        self.layernorm_after = nn.LayerNorm(d, eps=self.eps)
        self.mlp = _MLP(d, a["intermediate_size"])

    act = ACT_GELU_ERF  # ViTIntermediate: hidden_act "gelu" (exact erf)

    # role accessors shared with the CLIP layer (clip.py), which has other names
    @property
    def ln1(self):
        return self.layernorm_before

    @property
    def ln2(self):
        return self.layernorm_after

    @property
    def attn(self):
        return self.attention

    @property
    def fc1(self):
        return self.mlp.fc1

    @property
    def fc2(self):
        return self.mlp.fc2

    def forward(self, x, B, N):
        self.grad_graph = torch.is_grad_enabled()  # (inference: no act'(pre) kept, nothing saved)
        return _ViTLayerFn.apply(x, self.attn.o_proj.weight, self, B, N)


class _Pooler(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.dense = nn.Linear(d, d)


class CapkViTModel(CapkModule):
    """ViTModel (modeling_vit.py:336-381) with add_pooling_layer=True."""

    def __init__(self, arch):
        super().__init__()
        self.arch = dict(arch)
        self.config = type("ViTArch", (), dict(arch))()
        self.embeddings = _Embeddings(arch)
        self.layers = nn.ModuleList([ViTLayer(arch) for _ in range(arch["num_hidden_layers"])])
        self.layernorm = nn.LayerNorm(arch["hidden_size"], eps=arch["layer_norm_eps"])
        self.pooler = _Pooler(arch["hidden_size"])
        # backward links (not submodules): layer i's LN1 backward emits layer i-1's FC2 bias
        # gradient (the column sums of its dx), the head's final-LN backward the last layer's
        for prev, layer in zip(self.layers, self.layers[1:]):
            object.__setattr__(layer, "_capk_prev", prev)
        self._init_weights()

    def _init_weights(self):
        # ViTPreTrainedModel._init_weights: trunc-normal(0.02) weights, zero bias, LN 1/0
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                _trunc(m.weight.data)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        _trunc(self.embeddings.cls_token.data)
        _trunc(self.embeddings.position_embeddings.data)

    def _capk_optional_params(self):
        # the pooler receives no gradient when the decoder ignores pooled_features
        return [self.pooler.dense.weight, self.pooler.dense.bias]

    def forward(self, images):
        """images [B,C,H,W] -> (sequence_output [B*(N+1), D] flat, pooled [B, D])."""
        a = self.arch
        B = images.shape[0]
        P = a["patch_size"]
        Np = (images.shape[2] // P) * (images.shape[3] // P)
        N = Np + 1
        x = _ViTEmbedFn.apply(images, self.embeddings.patch_embeddings.projection.weight, self, B, Np)
        for layer in self.layers:
            x = layer(x, B, N)
        seq, pooled = _ViTHeadFn.apply(x, self.layernorm.weight, self, B, N)
        return seq, pooled


# --------------------------------------------------------------- functions --
class _ViTEmbedFn(torch.autograd.Function):
    """Patch conv as im2col + GEMM, then CLS + position embeddings (modeling_vit.py:60-69,129-161)."""

    @staticmethod
    def forward(ctx, images, anchor, m, B, Np):
        dt = m.cdtype
        P = m.arch["patch_size"]
        D = m.arch["hidden_size"]
        proj = m.embeddings.patch_embeddings.projection
        patches = ops.patchify(images, P, dt)
        pe = ops.linear(patches, W(proj.weight, dt).view(D, -1), proj.bias.detach())
        x = ops.vit_assemble(pe, m.embeddings.cls_token.detach(), m.embeddings.position_embeddings.detach(), B, Np,
                             D)
        ctx.m, ctx.B, ctx.Np = m, B, Np
        ctx.patches = patches
        return x

    @staticmethod
    def backward(ctx, dx):
        join_dw(dx.device)  # the layers' weight gradients (side stream) are complete from here on
        m, B, Np = ctx.m, ctx.B, ctx.Np
        D = m.arch["hidden_size"]
        dx = dx.contiguous()
        emb = m.embeddings
        dpatch = ops.vit_assemble_bwd(dx, B, Np, D, G(emb.cls_token).view(-1), G(emb.position_embeddings).view(-1))
        proj = emb.patch_embeddings.projection
        ops.linear_dw(dpatch, ctx.patches, G(proj.weight).view(D, -1))
        ops.colsum(dpatch, G(proj.bias))
        ctx.patches = None
        return None, None, None, None, None


class _ViTLayerFn(torch.autograd.Function):
    """Pre-LN encoder layer: ViTLayer.forward (modeling_vit.py:266-286) and, with the
    CLIP layer's accessors and quick_gelu, CLIPEncoderLayer.forward
    (modeling_clip.py:355-395)."""

    @staticmethod
    def forward(ctx, x, anchor, L, B, N):
        dt = L.cdtype
        D = x.shape[1]
        H = L.num_heads
        hd = D // H
        at, fc1, fc2, act = L.attn, L.fc1, L.fc2, L.act
        ln1, ln2 = L.ln1, L.ln2
        h1, mu1, rs1 = ops.layernorm_fwd(x, ln1.weight.detach(), ln1.bias.detach(), L.eps)
        qkv = ops.linear(h1, at.qkv_w.w(dt), at.qkv_b.master)
        o = torch.empty(x.shape[0], D, dtype=x.dtype, device=x.device)
        lse, _ = ops.attention_fwd(heads(qkv, 0, B, N), heads(qkv, D, B, N), heads(qkv, 2 * D, B, N),
                                   heads(o, 0, B, N), B, H, N, N, hd, 1.0 / math.sqrt(hd))
        x1 = ops.linear(o, W(at.o_proj.weight, dt), at.o_proj.bias.detach(), residual=x)
        h2, mu2, rs2 = ops.layernorm_fwd(x1, ln2.weight.detach(), ln2.bias.detach(), L.eps)
        I = fc1.weight.shape[0]
        if not getattr(L, "grad_graph", True):  # no_grad / inference (encoder of a beam search)
            f = ops.linear(h2, W(fc1.weight, dt), fc1.bias.detach(), act=act)
            return ops.linear(f, W(fc2.weight, dt), fc2.bias.detach(), residual=x1)
        f_pre = torch.empty(x.shape[0], I, dtype=x.dtype, device=x.device)
        # f_pre keeps act'(pre) (CAPK_ACT_DERIV): the FC1 epilogue writes GELU(pre) and its
        # derivative together, and the backward's dX epilogue multiplies by it and takes
        # FC1's bias gradient from the same registers (capk_gemm_dx_act_colsum)
        f = ops.linear(h2, W(fc1.weight, dt), fc1.bias.detach(), act=act | ACT_DERIV, preact=f_pre)
        y = ops.linear(f, W(fc2.weight, dt), fc2.bias.detach(), residual=x1)
        ctx.L, ctx.B, ctx.N = L, B, N
        ctx.saved = (x, h1, mu1, rs1, qkv, o, lse, x1, h2, mu2, rs2, f_pre, f)
        return y

    @staticmethod
    def backward(ctx, dy):
        L, B, N = ctx.L, ctx.B, ctx.N
        dt = L.cdtype
        x, h1, mu1, rs1, qkv, o, lse, x1, h2, mu2, rs2, f_pre, f = ctx.saved
        ctx.saved = None
        # the layer's LayerNorm / bias partial-sum finishes as one launch (ops.deferred_finishes)
        with ops.deferred_finishes():
            dy = dy.contiguous()
            D = x.shape[1]
            H = L.num_heads
            hd = D // H
            at, fc1, fc2, act = L.attn, L.fc1, L.fc2, L.act
            ln1, ln2 = L.ln1, L.ln2
            # FC2's bias gradient = colsum(dy): already produced by the LN backward that made dy
            # (next layer's LN1 / the head's final LN) when that one was linked to this layer
            fused_b2 = getattr(L, "_capk_fc2_bias_done", False)
            L._capk_fc2_bias_done = False
            # FC1's bias gradient = colsum(dfp), fused into the GELU' pass that produces dfp
            dfp = linear_bwd(dy, f, fc2.weight, None if fused_b2 else fc2.bias, dt, act_bwd=act | ACT_DERIV, aux=f_pre, side_dw=True,
                             dsum=G(fc1.bias))
            dh2 = linear_bwd(dfp, h2, fc1.weight, None, dt, side_dw=True)
            # dx1 = the O projection's output gradient: its column sums (O bias grad) come out of the LN kernel
            dx1 = ops.layernorm_bwd(dh2, x1, ln2.weight.detach(), mu2, rs2, G(ln2.weight), G(ln2.bias), dres=dy,
                                    dsum=G(at.o_proj.bias))
            do = linear_bwd(dx1, o, at.o_proj.weight, None, dt, side_dw=True)
            dqkv = torch.empty_like(qkv)
            hv = (heads(qkv, 0, B, N), heads(qkv, D, B, N), heads(qkv, 2 * D, B, N), heads(o, 0, B, N),
                  heads(do, 0, B, N), lse, heads(dqkv, 0, B, N), heads(dqkv, D, B, N), heads(dqkv, 2 * D, B, N),
                  B, H, N, N, hd, 1.0 / math.sqrt(hd))
            if _ATTN_BIAS:
                # the QKV bias gradient (column sums of dQ | dK | dV) comes out of the attention backward kernels
                ops.attention_bwd_bias(*hv, at.qkv_b.grad)
                dh1 = linear_bwd(dqkv, h1, None, None, dt, fused=(at.qkv_w, None), side_dw=True)
            else:
                ops.attention_bwd(*hv)
                dh1 = linear_bwd(dqkv, h1, None, None, dt, fused=(at.qkv_w, at.qkv_b), side_dw=True)
            prev = getattr(L, "_capk_prev", None)
            dx = ops.layernorm_bwd(dh1, x, ln1.weight.detach(), mu1, rs1, G(ln1.weight), G(ln1.bias), dres=dx1,
                                   dsum=G(prev.fc2.bias) if prev is not None else None)
            if prev is not None:
                prev._capk_fc2_bias_done = True
        notify_final(store_of(L), L.parameters())  # this layer's gradients are complete
        return dx, None, None, None, None


class _ViTHeadFn(torch.autograd.Function):
    """Final layernorm (modeling_vit.py:348) + ViTPooler tanh(dense(h[:,0])) (289-301)."""

    @staticmethod
    def forward(ctx, x, anchor, m, B, N):
        ctx.set_materialize_grads(False)
        dt = m.cdtype
        D = x.shape[1]
        ln = m.layernorm
        seq, mu, rs = ops.layernorm_fwd(x, ln.weight.detach(), ln.bias.detach(), ln.eps)
        cls_rows = seq.view(B, N, D)[:, 0]
        pre = torch.empty(B, D, dtype=seq.dtype, device=seq.device)
        dense = m.pooler.dense
        pooled = ops.linear(cls_rows, W(dense.weight, dt), dense.bias.detach(), act=ACT_TANH, preact=pre)
        ctx.m, ctx.B, ctx.N = m, B, N
        ctx.saved = (x, mu, rs, seq, pre)
        return seq, pooled

    @staticmethod
    def backward(ctx, dseq, dpooled):
        m, B, N = ctx.m, ctx.B, ctx.N
        dt = m.cdtype
        x, mu, rs, seq, pre = ctx.saved
        ctx.saved = None
        D = x.shape[1]
        if dseq is None:
            dseq = torch.zeros_like(seq)
        else:
            dseq = dseq.contiguous().clone() if dpooled is not None else dseq.contiguous()
        if dpooled is not None:
            dense = m.pooler.dense
            dpre = ops.act_bwd(dpooled.contiguous(), pre, ACT_TANH)
            cls_rows = seq.view(B, N, D)[:, 0]
            ops.linear_dw(dpre, cls_rows, G(dense.weight))
            ops.colsum(dpre, G(dense.bias))
            mark(dense.weight)
            mark(dense.bias)
            dcls = dseq.view(B, N, D)[:, 0]
            ops.linear_dx(dpre, W(dense.weight, dt), out=dcls, beta=1.0)
        ln = m.layernorm
        last = m.layers[-1] if len(m.layers) else None
        dx = ops.layernorm_bwd(dseq, x, ln.weight.detach(), mu, rs, G(ln.weight), G(ln.bias),
                               dsum=G(last.fc2.bias) if last is not None else None)
        if last is not None:
            last._capk_fc2_bias_done = True
        # the decoder and this head are done: everything but the embeddings and the layers is final
        notify_final(store_of(m), all_except=list(m.embeddings.parameters()) + list(m.layers.parameters()))
        return dx, None, None, None, None
