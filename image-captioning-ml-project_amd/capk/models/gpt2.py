"""GPT-2 caption decoder on libcapk kernels.

Restates src/models/decoders.py:495-656 (GPT2Decoder around transformers 5.15
``GPT2LMHeadModel``, modeling_gpt2.py:75-700) with the SURVEY D7 fix: the image
prefix ``P = image_to_prefix(pooled).view(B, 10, D)`` is every layer's cached
K = V (split into heads), the attention mask is ``cat(ones(B,10), captions != pad)``
and caption positions are 10..10+T-1.  Parameter names match the reference state
dict (``model.transformer.{wte,wpe,h.{i}.{ln_1,attn.c_attn,attn.c_proj,ln_2,mlp.c_fc,
mlp.c_proj},ln_f}``, tied ``model.lm_head``, ``visual_projection``, ``image_prefix``,
``image_to_prefix``); ``visual_projection`` and ``image_prefix`` are unused by the
reference forward (no gradient) and are skipped by AdamW like there.

Kernel mapping per block (pre-LN):
  LN -> c_attn Conv1D GEMM (weight [in,out] read N-major, no transpose) -> K/V rows of
  the captions gathered behind the 10 prefix rows -> attention (bottom-right causal
  over 10+T keys + key padding) -> c_proj GEMM (+bias, dropout, residual) -> LN ->
  c_fc GEMM (+bias, gelu_new, pre-activation kept) -> c_proj GEMM (+bias, dropout,
  residual); ln_f; LM head = GEMM against the (row-padded) tied wte.
Backward writes every gradient into the flat store; the tied wte receives the LM-head
gradient first and the embedding scatter-add on top; the prefix gradient is the sum
over layers of dK + dV of the prefix slots.
"""
import math
import os

import torch
import torch.nn as nn

from .. import ops
from .transformer import _history_reorder, _history_tables
from .._lib import ACT_DERIV, ACT_GELU_TANH
from ..ops import HeadView
from .common import G, CapkModule, W, heads, next_seed
from ..params import notify_final, store_of
from .transformer import _padded_grad, _pad64

PREFIX_LEN = 10  # decoders.py:540

GPT2_ARCHS = {
    "gpt2": dict(n_embd=768, n_layer=12, n_head=12, n_positions=1024, vocab_size=50257),
    "distilgpt2": dict(n_embd=768, n_layer=6, n_head=12, n_positions=1024, vocab_size=50257),
    "gpt2-medium": dict(n_embd=1024, n_layer=24, n_head=16, n_positions=1024, vocab_size=50257),
}


class _Conv1D(nn.Module):
    """transformers.pytorch_utils.Conv1D(nf, nx): weight [nx, nf], y = x @ W + b."""

    def __init__(self, nf, nx):
        super().__init__()
        self.nf = nf
        self.weight = nn.Parameter(torch.empty(nx, nf))
        self.bias = nn.Parameter(torch.zeros(nf))
        nn.init.normal_(self.weight, std=0.02)


class _GPT2Attention(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.c_attn = _Conv1D(3 * d, d)
        self.c_proj = _Conv1D(d, d)


class _GPT2MLP(nn.Module):
    def __init__(self, d, inner):
        super().__init__()
        self.c_fc = _Conv1D(inner, d)
        self.c_proj = _Conv1D(d, inner)


class _GPT2Block(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.ln_1 = nn.LayerNorm(d, eps=eps)
        self.attn = _GPT2Attention(d)
        self.ln_2 = nn.LayerNorm(d, eps=eps)
        self.mlp = _GPT2MLP(d, 4 * d)


class _GPT2Model(nn.Module):
    def __init__(self, c):
        super().__init__()
        d = c.n_embd
        self.wte = nn.Embedding(c.vocab_size, d)
        self.wpe = nn.Embedding(c.n_positions, d)
        self.h = nn.ModuleList([_GPT2Block(d, c.layer_norm_epsilon) for _ in range(c.n_layer)])
        self.ln_f = nn.LayerNorm(d, eps=c.layer_norm_epsilon)


class _GPT2LMHeadModel(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.config = c
        self.transformer = _GPT2Model(c)
        self.lm_head = nn.Linear(c.n_embd, c.vocab_size, bias=False)
        # GPT2PreTrainedModel._init_weights: normal(0.02), zero bias, LN 1/0, c_proj scaled by 1/sqrt(2L)
        for m in self.modules():
            if isinstance(m, nn.Embedding):
                nn.init.normal_(m.weight, std=0.02)
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        for blk in self.transformer.h:
            for cp in (blk.attn.c_proj, blk.mlp.c_proj):
                nn.init.normal_(cp.weight, std=0.02 / math.sqrt(2 * c.n_layer))
        self.lm_head.weight = self.transformer.wte.weight  # tie_word_embeddings


class GPT2Config:
    def __init__(self, vocab_size=50257, n_positions=1024, n_embd=768, n_layer=12, n_head=12, resid_pdrop=0.1,
                 embd_pdrop=0.1, attn_pdrop=0.1, layer_norm_epsilon=1e-5, **_):
        self.vocab_size, self.n_positions, self.n_embd = vocab_size, n_positions, n_embd
        self.n_layer, self.n_head = n_layer, n_head
        self.resid_pdrop, self.embd_pdrop, self.attn_pdrop = resid_pdrop, embd_pdrop, attn_pdrop
        self.layer_norm_epsilon = layer_norm_epsilon


class GPT2DecoderCore(CapkModule):
    """Compute core of capk.models.decoders.GPT2Decoder."""

    def __init__(self, config, vocab_size, pad_token_id, bos_token_id, eos_token_id):
        super().__init__()
        name = config.pretrained_model_name
        if name:
            if name not in GPT2_ARCHS:
                raise ValueError(f"capk GPT2Decoder: unknown architecture '{name}' (known: {sorted(GPT2_ARCHS)})")
            c = GPT2Config(**GPT2_ARCHS[name])
            if vocab_size:
                c.vocab_size = vocab_size  # resize_token_embeddings (decoders.py:515-518)
        else:  # decoders.py:520-531
            c = GPT2Config(vocab_size=vocab_size, n_positions=config.max_length, n_embd=config.hidden_dim,
                           n_layer=config.num_layers, n_head=config.num_heads, resid_pdrop=config.dropout,
                           embd_pdrop=config.dropout, attn_pdrop=config.dropout)
        self.model = _GPT2LMHeadModel(c)
        # decoders.py:534-536 (`or` defaults kept)
        self.pad_token_id = pad_token_id or 0
        self.bos_token_id = bos_token_id or 1
        self.eos_token_id = eos_token_id or 2
        d = c.n_embd
        self.visual_projection = nn.Linear(config.hidden_dim, d)
        self.prefix_length = PREFIX_LEN
        self.image_prefix = nn.Parameter(torch.randn(1, PREFIX_LEN, d))
        self.image_to_prefix = nn.Linear(config.hidden_dim, PREFIX_LEN * d)
        self.vocab_size = c.vocab_size
        self.vocab_pad = _pad64(c.vocab_size)
        self.model.transformer.wte.weight._capk_pad_rows = self.vocab_pad
        if PREFIX_LEN + 1 > c.n_positions:
            raise ValueError("capk GPT2Decoder: n_positions must exceed the 10-slot prefix")

    def _capk_optional_params(self):
        # unused by the reference forward: no gradient, AdamW skips them (torch: grad None)
        return [self.visual_projection.weight, self.visual_projection.bias, self.image_prefix]

    def _capk_store_first(self):
        # finished last by the backward (the prefix projection, after the embeddings): in front,
        # so ln_f and the blocks are a growing suffix for dp.GradBucketer (the tied wte -- LM
        # head and embedding -- is registered first already)
        return [self.image_to_prefix.weight, self.image_to_prefix.bias]

    def forward_logits(self, pooled, captions, use_pad_mask=True):
        """pooled [B, D], captions [B, T] int64 -> logits [B, T, V] (view of a padded buffer)."""
        return _GPT2Fn.apply(pooled, captions, self.model.transformer.wte.weight, self, use_pad_mask)


_IDX = {}


def _arange_i32(n, device):
    key = (n, str(device))
    t = _IDX.get(key)
    if t is None:
        t = _IDX[key] = torch.arange(n, dtype=torch.int32, device=device)
    return t


class _GPT2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pooled, captions, anchor, m, use_pad_mask):
        ctx.set_materialize_grads(False)
        dt = m.cdtype
        tr = m.model.transformer
        c = m.model.config
        B, T = captions.shape
        D, H = c.n_embd, c.n_head
        hd = D // H
        P = PREFIX_LEN
        Nk = P + T
        V, Vp = m.vocab_size, m.vocab_pad
        dev = captions.device
        captions = captions.contiguous()
        pooled = pooled.contiguous()
        if pooled.dtype != dt:
            raise TypeError(f"capk GPT2Decoder: pooled dtype {pooled.dtype} != compute dtype {dt}")
        if Nk > c.n_positions:
            raise ValueError(f"capk GPT2Decoder: 10 + T = {Nk} exceeds n_positions {c.n_positions}")
        itp = m.image_to_prefix
        prefix = ops.linear(pooled, W(itp.weight, dt), itp.bias.detach())  # [B, P*D]
        kp = None
        if use_pad_mask:  # D7: attention_mask = cat(ones(B,10), captions != pad)
            kp = torch.zeros(B, Nk, dtype=torch.uint8, device=dev)
            kp[:, P:] = (captions == m.pad_token_id)
        train = m.training
        seed = (lambda p: (p, next_seed())) if train else (lambda p: ops.NO_DROP)
        d_emb = seed(c.embd_pdrop)
        x = ops.embedding_fwd(captions, tr.wte.weight.detach(), tr.wpe.weight.detach(), P, dt, drop=d_emb)
        idxP, idxT = _arange_i32(P, dev), _arange_i32(T, dev)
        BT = B * T
        scale = 1.0 / math.sqrt(hd)
        saved = []
        for blk in tr.h:
            at, mlp = blk.attn, blk.mlp
            drops = (seed(c.attn_pdrop), seed(c.resid_pdrop), seed(c.resid_pdrop))
            x_in = x
            h1, mu1, rs1 = ops.layernorm_fwd(x, blk.ln_1.weight.detach(), blk.ln_1.bias.detach(), blk.ln_1.eps)
            qkv = ops.conv1d(h1, W(at.c_attn.weight, dt), at.c_attn.bias.detach())
            kvb = torch.empty(B * Nk, 2 * D, dtype=dt, device=dev)
            # prefix rows: K = V = P (D7); caption rows: this layer's K/V
            ops.gather_rows(prefix, idxP, kvb, B, P, D, D, P * D, 2 * D, Nk * 2 * D)
            ops.gather_rows(prefix, idxP, kvb, B, P, D, D, P * D, 2 * D, Nk * 2 * D, y_off=D)
            ops.gather_rows(qkv, idxT, kvb, B, T, 2 * D, 3 * D, T * 3 * D, 2 * D, Nk * 2 * D, x_off=D, y_off=P * 2 * D)
            a = torch.empty(BT, D, dtype=dt, device=dev)
            kview, vview = HeadView(kvb, 0, Nk * 2 * D, 2 * D), HeadView(kvb, D, Nk * 2 * D, 2 * D)
            lse, kpu = ops.attention_fwd(heads(qkv, 0, B, T), kview, vview, heads(a, 0, B, T), B, H, T, Nk, hd, scale,
                                         causal=True, key_pad=kp, drop=drops[0])
            x1 = ops.conv1d(a, W(at.c_proj.weight, dt), at.c_proj.bias.detach(), residual=x, drop=drops[1])
            h2, mu2, rs2 = ops.layernorm_fwd(x1, blk.ln_2.weight.detach(), blk.ln_2.bias.detach(), blk.ln_2.eps)
            I = mlp.c_fc.weight.shape[1]
            f_pre = torch.empty(BT, I, dtype=dt, device=dev)
            f = ops.conv1d(h2, W(mlp.c_fc.weight, dt), mlp.c_fc.bias.detach(), act=ACT_GELU_TANH | ACT_DERIV, preact=f_pre)
            x = ops.conv1d(f, W(mlp.c_proj.weight, dt), mlp.c_proj.bias.detach(), residual=x1, drop=drops[2])
            saved.append((x_in, h1, mu1, rs1, qkv, kvb, a, lse, kpu, x1, h2, mu2, rs2, f_pre, f, drops))
        xf, muf, rsf = ops.layernorm_fwd(x, tr.ln_f.weight.detach(), tr.ln_f.bias.detach(), tr.ln_f.eps)
        wte = tr.wte.weight
        wout = wte._capk_pad_bf16 if dt == torch.bfloat16 else wte._capk_pad_master
        logits_pad = ops.linear(xf, wout, None)
        ctx.m, ctx.d_emb = m, d_emb
        ctx.dims = (B, T, D, H, hd, P, Nk, V, Vp, scale)
        ctx.saved = (pooled, captions, prefix, saved, x, muf, rsf, xf)
        ctx.logits_pad = logits_pad
        return logits_pad[:, :V].view(B, T, V)

    @staticmethod
    def backward(ctx, dlogits):
        m = ctx.m
        dt = m.cdtype
        tr = m.model.transformer
        B, T, D, H, hd, P, Nk, V, Vp, scale = ctx.dims
        pooled, captions, prefix, saved, xL, muf, rsf, xf = ctx.saved
        ctx.saved = None
        dev = xf.device
        BT = B * T
        wte = tr.wte.weight
        wout = wte._capk_pad_bf16 if dt == torch.bfloat16 else wte._capk_pad_master
        idxT = _arange_i32(T, dev)
        if dlogits is None:
            ops.zero_(wte._capk_pad_grad)
            dxf = torch.zeros(BT, D, dtype=dt, device=dev)
        else:
            dl = _padded_grad(dlogits, ctx.logits_pad, BT, V, Vp)
            ops.linear_dw(dl, xf, wte._capk_pad_grad)  # tied LM head: written first (beta 0)
            dxf = ops.linear_dx(dl, wout)
        ctx.logits_pad = None
        dx = ops.layernorm_bwd(dxf, xL, tr.ln_f.weight.detach(), muf, rsf, G(tr.ln_f.weight), G(tr.ln_f.bias))
        store = store_of(m)
        notify_final(store, [tr.ln_f.weight, tr.ln_f.bias])
        dprefix = torch.empty(B, P * D, dtype=torch.float32, device=dev)
        for li in range(len(saved) - 1, -1, -1):
            blk = tr.h[li]
            at, mlp = blk.attn, blk.mlp
            (x_in, h1, mu1, rs1, qkv, kvb, a, lse, kpu, x1, h2, mu2, rs2, f_pre, f, drops) = saved[li]
            saved[li] = None
            # x = x1 + drop(c_proj(gelu_new(c_fc(ln_2 x1))))
            dym = ops.dropout_apply(dx, drops[2])
            dfp = ops.conv1d_dx(dym, W(mlp.c_proj.weight, dt), act_bwd=ACT_GELU_TANH | ACT_DERIV, aux=f_pre)
            ops.linear_dw(f, dym, G(mlp.c_proj.weight))
            ops.colsum(dym, G(mlp.c_proj.bias))
            dh2 = ops.conv1d_dx(dfp, W(mlp.c_fc.weight, dt))
            ops.linear_dw(h2, dfp, G(mlp.c_fc.weight))
            ops.colsum(dfp, G(mlp.c_fc.bias))
            dx1 = ops.layernorm_bwd(dh2, x1, blk.ln_2.weight.detach(), mu2, rs2, G(blk.ln_2.weight), G(blk.ln_2.bias),
                                    dres=dx)
            # x1 = x + drop(c_proj(attn(ln_1 x)))
            dx1m = ops.dropout_apply(dx1, drops[1])
            da = ops.conv1d_dx(dx1m, W(at.c_proj.weight, dt))
            ops.linear_dw(a, dx1m, G(at.c_proj.weight))
            ops.colsum(dx1m, G(at.c_proj.bias))
            dqkv = torch.empty(BT, 3 * D, dtype=dt, device=dev)
            dkvb = torch.empty(B * Nk, 2 * D, dtype=dt, device=dev)
            ops.attention_bwd(heads(qkv, 0, B, T), HeadView(kvb, 0, Nk * 2 * D, 2 * D),
                              HeadView(kvb, D, Nk * 2 * D, 2 * D), heads(a, 0, B, T), heads(da, 0, B, T), lse,
                              heads(dqkv, 0, B, T), HeadView(dkvb, 0, Nk * 2 * D, 2 * D),
                              HeadView(dkvb, D, Nk * 2 * D, 2 * D), B, H, T, Nk, hd, scale, causal=True,
                              key_pad_u8=kpu, drop=drops[0])
            ops.gather_rows(dkvb, idxT, dqkv, B, T, 2 * D, 2 * D, Nk * 2 * D, 3 * D, T * 3 * D, x_off=P * 2 * D,
                            y_off=D)
            # prefix slots: dP += dK + dV (same P in every layer)
            ops.add_rows(dkvb, dprefix, B, P, D, Nk * 2 * D, 2 * D, 2, D, P * D, D, accumulate=li != len(saved) - 1)
            dh1 = ops.conv1d_dx(dqkv, W(at.c_attn.weight, dt))
            ops.linear_dw(h1, dqkv, G(at.c_attn.weight))
            ops.colsum(dqkv, G(at.c_attn.bias))
            dx = ops.layernorm_bwd(dh1, x_in, blk.ln_1.weight.detach(), mu1, rs1, G(blk.ln_1.weight),
                                   G(blk.ln_1.bias), dres=dx1)
            notify_final(store, blk.parameters())  # this block's gradients are complete
        # embeddings: wte already holds the LM-head gradient; wpe rows 10..10+T-1
        ops.zero_(G(tr.wpe.weight))
        ops.embedding_bwd(captions, dx, None, G(wte), G(tr.wpe.weight), P, drop=ctx.d_emb)
        # prefix -> image_to_prefix -> pooled
        itp = m.image_to_prefix
        dP = dprefix if dt == torch.float32 else torch.empty(B, P * D, dtype=dt, device=dev)
        if dt != torch.float32:
            ops.cast(dprefix, dP)
        ops.linear_dw(dP, pooled, G(itp.weight))
        ops.colsum(dP, G(itp.bias))
        notify_final(store, [wte, tr.wpe.weight, itp.weight, itp.bias])
        dpooled = ops.linear_dx(dP, W(itp.weight, dt))
        return dpooled, None, None, None, None


class GPT2KVRunner:
    """KV-cached incremental decode of the D7-restated GPT-2 for beam search: per layer
    a cache [B*k, 10 + max_length, 3D] whose first 10 rows hold K = V = the image's
    prefix (copied per beam once), then one row per generated position written by the
    c_attn GEMM; self-attention of the new token reads rows 0..10+t in place
    (decode kernel); caches of all layers are reordered in one gather launch per step
    (HF Cache.reorder_cache).  Positions are 10 + t (modeling_gpt2.py:569-574)."""

    def __init__(self, m, pooled, num_beams, max_length):
        dt = m.cdtype
        c = m.model.config
        self.m, self.dt, self.k = m, dt, num_beams
        B = pooled.shape[0]
        D, H = c.n_embd, c.n_head
        self.B, self.D, self.H, self.hd = B, D, H, D // H
        self.scale = 1.0 / math.sqrt(self.hd)
        P = PREFIX_LEN
        self.P, self.Lc = P, P + max_length
        if P + max_length > c.n_positions:
            raise ValueError(f"capk GPT2 generate: 10 + max_length exceeds n_positions {c.n_positions}")
        dev = pooled.device
        R = B * num_beams
        self.R = R
        shape = (c.n_layer, R, self.Lc, 3 * D)
        # beam-history table instead of a reordered cache (transformer.KVDecodeRunner);
        # CAPK_KV_GATHER=1: the whole-cache gather with ping-pong buffers
        self.gather_kv = os.environ.get("CAPK_KV_GATHER", "0") == "1"
        self._bufs = (torch.empty(shape, dtype=dt, device=dev),
                      torch.empty(shape, dtype=dt, device=dev) if self.gather_kv else None)
        self.hist, self.hist_tmp, self.hist0 = _history_tables(R, self.Lc, dev)
        self.pref_rep = torch.empty(R, P * D, dtype=dt, device=dev)
        self.rep_idx = torch.arange(R, dtype=torch.int32, device=dev) // num_beams
        wte = m.model.transformer.wte.weight
        self.wout = wte._capk_pad_bf16 if dt == torch.bfloat16 else wte._capk_pad_master
        self.load(pooled)

    def load(self, pooled):
        """Per-call state, written in place (a runner reused by capk.graphs keeps its buffers):
        the image prefix into the K/V slots of the first 10 rows of every layer's cache."""
        m, dt, P, D, R = self.m, self.dt, self.P, self.D, self.R
        if pooled.dtype != dt:
            raise TypeError(f"capk GPT2Decoder: pooled dtype {pooled.dtype} != compute dtype {dt}")
        if pooled.shape[0] != self.B:
            raise ValueError("capk GPT2KVRunner.load: batch size differs from the runner's")
        itp = m.image_to_prefix
        prefix = ops.linear(pooled.contiguous(), W(itp.weight, dt), itp.bias.detach())  # [B, P*D]
        ops.gather_rows(prefix, self.rep_idx, self.pref_rep, 1, R, P * D, P * D, 0, P * D, 0)
        self.reset()
        idxP = _arange_i32(P, pooled.device)
        Lc3 = self.Lc * 3 * D
        for li in range(self.cache.shape[0]):
            for slot in (1, 2):  # K and V slots of the prefix rows
                ops.gather_rows(self.pref_rep, idxP, self.cache[li], R, P, D, D, P * D, 3 * D, Lc3, y_off=slot * D)

    def reset(self):
        self.cache, self.spare = self._bufs
        self.hist.copy_(self.hist0)

    def step(self, cur_len, ids, reorder_idx):
        m, dt, D, H, hd, R, P = self.m, self.dt, self.D, self.H, self.hd, self.R, self.P
        tr = m.model.transformer
        t = cur_len - 1
        pos = P + t
        Lc3 = self.Lc * 3 * D
        if reorder_idx is not None:
            if self.gather_kv:
                c = self.cache
                nl = c.shape[0]
                ops.gather_rows(c, reorder_idx, self.spare, nl, R, pos * 3 * D, Lc3, R * Lc3, Lc3, R * Lc3)
                self.cache, self.spare = self.spare, self.cache
            else:  # (the 10 prefix positions are the same row content for every beam of an image)
                _history_reorder(self.hist, self.hist_tmp, reorder_idx, pos)
        x = ops.embedding_fwd(ids.view(R, 1), tr.wte.weight.detach(), tr.wpe.weight.detach(), pos, dt)
        # the MLP projection of block l is summed by block l+1's ln_1 (ln_f after the last),
        # the attention projection by ln_2 (ops.product_ln: split-K slabs read by the LayerNorm)
        mlp_out = None  # (f, W, bias, residual) of the previous block's MLP projection
        for li, blk in enumerate(tr.h):
            at, mlp = blk.attn, blk.mlp
            cl = self.cache[li]
            if mlp_out is None:
                h1, _, _ = ops.layernorm_fwd(x, blk.ln_1.weight.detach(), blk.ln_1.bias.detach(), blk.ln_1.eps)
            else:
                h1, x = ops.product_ln(*mlp_out, blk.ln_1.weight.detach(), blk.ln_1.bias.detach(), blk.ln_1.eps,
                                       keep=True)
            ops.conv1d(h1, W(at.c_attn.weight, dt), at.c_attn.bias.detach(), out=cl[:, pos, :])
            a = torch.empty(R, D, dtype=dt, device=x.device)
            qv, kv_, vv = HeadView(cl, pos * 3 * D, Lc3, 3 * D), HeadView(cl, D, Lc3, 3 * D), HeadView(cl, 2 * D, Lc3, 3 * D)
            if self.gather_kv:
                ops.attention_fwd(qv, kv_, vv, HeadView(a, 0, D, D), R, H, 1, pos + 1, hd, self.scale)
            else:
                ops.attention_decode_rows(qv, kv_, vv, HeadView(a, 0, D, D), self.hist, R, H, 1, pos + 1, hd,
                                          self.scale)
            h2, x1 = ops.product_ln(a, W(at.c_proj.weight, dt), True, at.c_proj.bias.detach(), x,
                                    blk.ln_2.weight.detach(), blk.ln_2.bias.detach(), blk.ln_2.eps, keep=True)
            f = ops.conv1d(h2, W(mlp.c_fc.weight, dt), mlp.c_fc.bias.detach(), act=ACT_GELU_TANH)
            mlp_out = (f, W(mlp.c_proj.weight, dt), True, mlp.c_proj.bias.detach(), x1)
        xf, _ = ops.product_ln(*mlp_out, tr.ln_f.weight.detach(), tr.ln_f.bias.detach(), tr.ln_f.eps)
        return ops.linear(xf, self.wout, None)
