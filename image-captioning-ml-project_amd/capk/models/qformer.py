"""BLIP-2 style Q-Former on libcapk kernels — mirrors the reference's
``QFormer`` (src/models/captioning_model.py:153-245) and its use in
``ImageCaptioningModel.forward`` / ``generate`` (captioning_model.py:79-91,130-141).

Parameter names are the reference state dict's: ``query_tokens``, ``vision_proj``
(Identity when vision_dim == query_dim), ``encoder.layers.{i}`` (norm_first
``nn.TransformerEncoderLayer``: ``self_attn.in_proj_weight/bias``, ``self_attn.out_proj``,
``linear1``, ``linear2``, ``norm1``, ``norm2``) and ``decoder.layers.{i}`` (norm_first
``nn.TransformerDecoderLayer``: + ``multihead_attn``, ``norm3``).

Kernel mapping (one autograd Function for the whole module, dropout sites of torch's
layers in train mode):
  queries broadcast (gather) -> encoder blocks: LN -> packed QKV GEMM -> attention (Q x Q,
  probability dropout) -> out-proj GEMM (+bias, dropout1, residual) -> LN -> FC1 GEMM
  (+bias, GELU, dropout) -> FC2 GEMM (+bias, dropout2, residual)
  -> decoder blocks: the same self-attention branch, then LN -> Q GEMM, K/V GEMM of the
  vision features (+ CLS-row gaps addressed, not copied) -> attention (Q x S) -> out-proj
  (+residual), then the FFN branch.
The vision features' attention mask (all ones from every capk encoder) is the additive 0
mask of the reference (captioning_model.py:225-227): no key masking.
"""
import math

import torch
import torch.nn as nn

from .. import ops
from .._lib import ACT_DERIV, ACT_GELU_ERF
from ..ops import HeadView
from .common import G, CapkModule, W, heads, linear_bwd, next_seed
from .transformer import _mem_geometry


class _MHA(nn.Module):
    """nn.MultiheadAttention parameter layout (packed in_proj)."""

    def __init__(self, d):
        super().__init__()
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.out_proj = nn.Linear(d, d)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)


class QFormerEncoderLayer(nn.Module):
    def __init__(self, d, ff):
        super().__init__()
        self.self_attn = _MHA(d)
        self.linear1 = nn.Linear(d, ff)
        self.linear2 = nn.Linear(ff, d)
        self.norm1 = nn.LayerNorm(d)
        self.norm2 = nn.LayerNorm(d)


class QFormerDecoderLayer(QFormerEncoderLayer):
    def __init__(self, d, ff):
        super().__init__(d, ff)
        self.multihead_attn = _MHA(d)
        self.norm3 = nn.LayerNorm(d)


class _Stack(nn.Module):
    def __init__(self, layers):
        super().__init__()
        self.layers = nn.ModuleList(layers)


class QFormer(CapkModule):
    """captioning_model.py:153-245 (same constructor arguments)."""

    def __init__(self, query_dim=768, vision_dim=768, num_queries=32, num_layers=2, num_heads=8, dropout=0.1):
        super().__init__()
        if query_dim % num_heads:
            raise ValueError("capk QFormer: query_dim must be divisible by num_heads")
        self.query_tokens = nn.Parameter(torch.zeros(1, num_queries, query_dim))
        nn.init.normal_(self.query_tokens, std=0.02)
        self.vision_proj = nn.Linear(vision_dim, query_dim) if vision_dim != query_dim else nn.Identity()
        self.encoder = _Stack([QFormerEncoderLayer(query_dim, 4 * query_dim) for _ in range(num_layers)])
        self.decoder = _Stack([QFormerDecoderLayer(query_dim, 4 * query_dim) for _ in range(num_layers)])
        self.num_heads, self.num_queries, self.dropout_p = num_heads, num_queries, dropout

    def forward(self, vision_features, vision_attention_mask=None):
        """vision_features [B, S, vision_dim] (rows contiguous, batch stride may exceed S
        rows) -> {"queries": [B, num_queries, query_dim]}."""
        for p in self.parameters():
            self._check_ready(p)
        q = _QFormerFn.apply(vision_features, self.query_tokens, self)
        return {"queries": q}


class _QFormerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, features, anchor, m):
        dt = m.cdtype
        B, S, Dv = features.shape
        Q, D = m.num_queries, m.query_tokens.shape[-1]
        H = m.num_heads
        hd = D // H
        scale = 1.0 / math.sqrt(hd)
        if features.dtype != dt:
            raise TypeError(f"capk QFormer: features dtype {features.dtype} != compute dtype {dt}")
        dev = features.device
        feat_mem, rpb, M_ext = _mem_geometry(features)
        if isinstance(m.vision_proj, nn.Linear):
            mem = ops.linear(feat_mem, W(m.vision_proj.weight, dt), m.vision_proj.bias.detach())
        else:
            mem = feat_mem
        p = m.dropout_p if m.training else 0.0
        seed = (lambda: (p, next_seed())) if p > 0 else (lambda: ops.NO_DROP)
        BQ = B * Q
        x = torch.empty(BQ, D, dtype=dt, device=dev)
        idx = torch.arange(Q, dtype=torch.int32, device=dev)
        ops.gather_rows(W(m.query_tokens, dt).view(Q, D), idx, x, B, Q, D, D, 0, D, Q * D)

        def self_attn_branch(L, x, drops):
            h1, mu1, rs1 = ops.layernorm_fwd(x, L.norm1.weight.detach(), L.norm1.bias.detach(), L.norm1.eps)
            sa = L.self_attn
            qkv = ops.linear(h1, W(sa.in_proj_weight, dt), sa.in_proj_bias.detach())
            a = torch.empty(BQ, D, dtype=dt, device=dev)
            lse, _ = ops.attention_fwd(heads(qkv, 0, B, Q), heads(qkv, D, B, Q), heads(qkv, 2 * D, B, Q),
                                       heads(a, 0, B, Q), B, H, Q, Q, hd, scale, drop=drops[0])
            x1 = ops.linear(a, W(sa.out_proj.weight, dt), sa.out_proj.bias.detach(), residual=x, drop=drops[1])
            return x1, (h1, mu1, rs1, qkv, a, lse)

        def ffn_branch(L, x, norm, drops):
            h, mu, rs = ops.layernorm_fwd(x, norm.weight.detach(), norm.bias.detach(), norm.eps)
            I = L.linear1.weight.shape[0]
            f_pre = torch.empty(BQ, I, dtype=dt, device=dev)
            f = ops.linear(h, W(L.linear1.weight, dt), L.linear1.bias.detach(), act=ACT_GELU_ERF | ACT_DERIV,
                           preact=f_pre, drop=drops[0])
            y = ops.linear(f, W(L.linear2.weight, dt), L.linear2.bias.detach(), residual=x, drop=drops[1])
            return y, (h, mu, rs, f_pre, f)

        saved_enc, saved_dec = [], []
        for L in m.encoder.layers:
            drops = tuple(seed() for _ in range(4))  # attn prob, dropout1, ffn inner, dropout2
            x_in = x
            x1, sa_s = self_attn_branch(L, x, drops[0:2])
            x, ff_s = ffn_branch(L, x1, L.norm2, drops[2:4])
            saved_enc.append((x_in, x1, sa_s, ff_s, drops))
        for L in m.decoder.layers:
            drops = tuple(seed() for _ in range(6))  # sa prob, dropout1, ca prob, dropout2, ffn inner, dropout3
            x_in = x
            x1, sa_s = self_attn_branch(L, x, drops[0:2])
            h2, mu2, rs2 = ops.layernorm_fwd(x1, L.norm2.weight.detach(), L.norm2.bias.detach(), L.norm2.eps)
            ca = L.multihead_attn
            wca, bca = W(ca.in_proj_weight, dt), ca.in_proj_bias.detach()
            qc = ops.linear(h2, wca[:D], bca[:D])
            kv = ops.linear(mem, wca[D:], bca[D:])  # [M_ext, 2D]
            c = torch.empty(BQ, D, dtype=dt, device=dev)
            lse2, _ = ops.attention_fwd(heads(qc, 0, B, Q), HeadView(kv, 0, rpb * 2 * D, 2 * D),
                                        HeadView(kv, D, rpb * 2 * D, 2 * D), heads(c, 0, B, Q), B, H, Q, S, hd,
                                        scale, drop=drops[2])
            x2 = ops.linear(c, W(ca.out_proj.weight, dt), ca.out_proj.bias.detach(), residual=x1, drop=drops[3])
            x, ff_s = ffn_branch(L, x2, L.norm3, drops[4:6])
            saved_dec.append((x_in, x1, sa_s, (h2, mu2, rs2, qc, kv, c, lse2), x2, ff_s, drops))
        ctx.m = m
        ctx.dims = (B, S, Q, D, H, hd, scale, rpb, M_ext, BQ)
        ctx.saved = (feat_mem, mem, saved_enc, saved_dec)
        ctx.features_meta = (features.shape, features.stride())
        return x.view(B, Q, D)

    @staticmethod
    def backward(ctx, dout):
        m = ctx.m
        dt = m.cdtype
        B, S, Q, D, H, hd, scale, rpb, M_ext, BQ = ctx.dims
        feat_mem, mem, saved_enc, saved_dec = ctx.saved
        ctx.saved = None
        dev = feat_mem.device
        dx = dout.reshape(BQ, D).to(dt).contiguous()

        def ffn_bwd(L, dy, x, norm, s, drops):
            """y = x + drop2(W2 drop(GELU(W1 LN(x)))) -> dx."""
            h, mu, rs, f_pre, f = s
            dym = ops.dropout_apply(dy, drops[1])
            dfp = linear_bwd(dym, f, L.linear2.weight, L.linear2.bias, dt, act_bwd=ACT_GELU_ERF | ACT_DERIV, aux=f_pre,
                             drop=drops[0])
            dh = linear_bwd(dfp, h, L.linear1.weight, L.linear1.bias, dt)
            return ops.layernorm_bwd(dh, x, norm.weight.detach(), mu, rs, G(norm.weight), G(norm.bias), dres=dy)

        def sa_bwd(L, dy, x, s, drops):
            """y = x + drop1(Wo attn(LN1 x)) -> dx."""
            h1, mu1, rs1, qkv, a, lse = s
            sa = L.self_attn
            dym = ops.dropout_apply(dy, drops[1])
            da = linear_bwd(dym, a, sa.out_proj.weight, sa.out_proj.bias, dt)
            dqkv = torch.empty_like(qkv)
            ops.attention_bwd(heads(qkv, 0, B, Q), heads(qkv, D, B, Q), heads(qkv, 2 * D, B, Q), heads(a, 0, B, Q),
                              heads(da, 0, B, Q), lse, heads(dqkv, 0, B, Q), heads(dqkv, D, B, Q),
                              heads(dqkv, 2 * D, B, Q), B, H, Q, Q, hd, scale, drop=drops[0])
            dh1 = linear_bwd(dqkv, h1, sa.in_proj_weight, sa.in_proj_bias, dt)
            return ops.layernorm_bwd(dh1, x, L.norm1.weight.detach(), mu1, rs1, G(L.norm1.weight), G(L.norm1.bias),
                                     dres=dy)

        dmem = None
        for li in range(len(saved_dec) - 1, -1, -1):
            L = m.decoder.layers[li]
            x_in, x1, sa_s, ca_s, x2, ff_s, drops = saved_dec[li]
            saved_dec[li] = None
            dx2 = ffn_bwd(L, dx, x2, L.norm3, ff_s, drops[4:6])
            h2, mu2, rs2, qc, kv, c, lse2 = ca_s
            ca = L.multihead_attn
            dx2m = ops.dropout_apply(dx2, drops[3])
            dc = linear_bwd(dx2m, c, ca.out_proj.weight, ca.out_proj.bias, dt)
            dqc = torch.empty(BQ, D, dtype=dt, device=dev)
            dkv = torch.empty(M_ext, 2 * D, dtype=dt, device=dev)
            if rpb != S:
                ops.zero_(dkv)  # gap rows (e.g. the ViT CLS rows) get no K/V gradient
            ops.attention_bwd(heads(qc, 0, B, Q), HeadView(kv, 0, rpb * 2 * D, 2 * D),
                              HeadView(kv, D, rpb * 2 * D, 2 * D), heads(c, 0, B, Q), heads(dc, 0, B, Q), lse2,
                              heads(dqc, 0, B, Q), HeadView(dkv, 0, rpb * 2 * D, 2 * D),
                              HeadView(dkv, D, rpb * 2 * D, 2 * D), B, H, Q, S, hd, scale, drop=drops[2])
            gW, gB = G(ca.in_proj_weight), G(ca.in_proj_bias)
            wca = W(ca.in_proj_weight, dt)
            ops.linear_dw(dkv, mem, gW[D:])
            ops.colsum(dkv, gB[D:])
            if dmem is None:
                dmem = ops.linear_dx(dkv, wca[D:])
            else:
                ops.linear_dx(dkv, wca[D:], out=dmem, beta=1.0)
            ops.linear_dw(dqc, h2, gW[:D])
            ops.colsum(dqc, gB[:D])
            dh2 = ops.linear_dx(dqc, wca[:D])
            dx1 = ops.layernorm_bwd(dh2, x1, L.norm2.weight.detach(), mu2, rs2, G(L.norm2.weight), G(L.norm2.bias),
                                    dres=dx2)
            dx = sa_bwd(L, dx1, x_in, sa_s, drops[0:2])
        for li in range(len(saved_enc) - 1, -1, -1):
            L = m.encoder.layers[li]
            x_in, x1, sa_s, ff_s, drops = saved_enc[li]
            saved_enc[li] = None
            dx1 = ffn_bwd(L, dx, x1, L.norm2, ff_s, drops[2:4])
            dx = sa_bwd(L, dx1, x_in, sa_s, drops[0:2])
        # queries: d query_tokens = sum over the batch of the rows' gradients
        ops.colsum(dx.view(B, Q * D), G(m.query_tokens).view(-1))
        if dmem is None:  # no decoder layers
            dmem = torch.zeros(M_ext, D, dtype=dt, device=dev)
        if isinstance(m.vision_proj, nn.Linear):
            vp = m.vision_proj
            ops.linear_dw(dmem, feat_mem, G(vp.weight))
            ops.colsum(dmem, G(vp.bias))
            dfeat = ops.linear_dx(dmem, W(vp.weight, dt))
        else:
            dfeat = dmem
        shape, stride = ctx.features_meta
        return dfeat.as_strided(shape, stride, 0), None, None
