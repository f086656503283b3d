"""Transformer caption decoder on libcapk kernels.

Restates src/models/decoders.py:317-493 (TransformerDecoder) whose layers are
torch ``nn.TransformerDecoderLayer`` (post-LN, GELU, batch_first;
torch/nn/modules/transformer.py:985-1200).  Parameter names are identical to
the reference state dict (``embedding``, ``position_encoding``,
``transformer_decoder.layers.{i}.self_attn.in_proj_weight`` ..., ``output_layer``,
``visual_projection``).

The whole teacher-forced pass — token+position embedding, N post-LN layers,
LM head — is ONE autograd Function, so the memory gradient shared by all
cross-attention K/V projections is accumulated in place by beta=1 GEMM
epilogues instead of by autograd adds.  The vocabulary dimension of the LM
head is zero-padded to a multiple of 64 (``Vp``) inside the flat parameter
store, so every LM-head GEMM runs on full tiles; the returned logits are a
[B, T, V] view of the padded [B*T, Vp] buffer.

Memory features may come with a row gap per batch element (the ViT sequence
output minus its CLS row is a strided view): the K/V projection runs on the
underlying rows and attention addresses batch b at row b*(S+gap) — no copy.
"""
import copy
import math
import os

import torch
import torch.nn as nn

from .. import ops
from .._lib import ACT_DERIV, ACT_GELU_ERF
from .common import G, CapkModule, W, heads, linear_bwd, next_seed
from ..ops import HeadView
from ..params import notify_final, store_of


def _pad64(v):
    return (v + 63) // 64 * 64


class _DecoderLayerParams(nn.Module):
    """Parameter holder with nn.TransformerDecoderLayer's names (and its init)."""

    def __init__(self, d, nhead, dff, dropout):
        super().__init__()
        ref = nn.TransformerDecoderLayer(d, nhead, dff, dropout, activation="gelu", batch_first=True)
        self.self_attn = ref.self_attn
        self.multihead_attn = ref.multihead_attn
        self.linear1 = ref.linear1
        self.linear2 = ref.linear2
        self.norm1 = ref.norm1
        self.norm2 = ref.norm2
        self.norm3 = ref.norm3
        self.nhead = nhead
        self.dropout_p = dropout


class _TransformerDecoderStack(nn.Module):
    def __init__(self, layer, num_layers):
        super().__init__()
        # nn.TransformerDecoder deep-copies one layer: every layer starts from identical weights
        self.layers = nn.ModuleList([copy.deepcopy(layer) for _ in range(num_layers)])
        self.num_layers = num_layers


class TransformerDecoderCore(CapkModule):
    """Compute core used by capk.models.decoders.TransformerDecoder."""

    def __init__(self, hidden_dim, num_layers, num_heads, dropout, max_length, vocab_size, pad_token_id):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.num_heads = num_heads
        self.vocab_size = vocab_size
        self.vocab_pad = _pad64(vocab_size)
        self.pad_token_id = pad_token_id
        self.dropout_p = dropout
        self.embedding = nn.Embedding(vocab_size, hidden_dim, padding_idx=pad_token_id)
        self.position_encoding = nn.Embedding(max_length, hidden_dim)
        layer = _DecoderLayerParams(hidden_dim, num_heads, hidden_dim * 4, dropout)
        self.transformer_decoder = _TransformerDecoderStack(layer, num_layers)
        self.output_layer = nn.Linear(hidden_dim, vocab_size)
        self.visual_projection = nn.Linear(hidden_dim, hidden_dim)
        self.output_layer.weight._capk_pad_rows = self.vocab_pad
        self.output_layer.bias._capk_pad_rows = self.vocab_pad

    def _capk_store_first(self):
        # the backward finishes the visual projection last (after the embeddings): in front of
        # the embeddings in the flat buffers, so the LM head and every layer are a growing
        # suffix that dp.GradBucketer exchanges while the rest of the backward runs
        return [self.visual_projection.weight, self.visual_projection.bias]

    # -------------------------------------------------------------- forward
    def forward_logits(self, features, captions, use_pad_mask=True):
        """features [B,S,D] (row stride may include a gap), captions [B,T] int64 ->
        (logits [B,T,V] view, hidden [B,T,D]).  use_pad_mask: tgt_key_padding_mask =
        captions == pad (decoders.py:405); generate() passes none (decoders.py:473-477)."""
        return _DecoderFn.apply(features, captions, self.visual_projection.weight, self, use_pad_mask)


def _mem_geometry(features):
    """Rows of the memory as a [M_ext, D] matrix over the features' own storage."""
    B, S, D = features.shape
    assert features.stride(2) == 1 and features.stride(1) == D, "features rows must be contiguous"
    rows_per_b = features.stride(0) // D
    assert features.stride(0) % D == 0 and rows_per_b >= S
    M_ext = (B - 1) * rows_per_b + S
    mem = features.as_strided((M_ext, D), (D, 1))
    return mem, rows_per_b, M_ext


class _DecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, features, captions, anchor, m, use_pad_mask):
        ctx.set_materialize_grads(False)
        dt = m.cdtype
        B, S, D = features.shape
        T = captions.shape[1]
        H = m.num_heads
        hd = D // H
        scale = 1.0 / math.sqrt(hd)
        V, Vp = m.vocab_size, m.vocab_pad
        captions = captions.contiguous()
        if features.dtype != dt:
            raise TypeError(f"capk TransformerDecoder: features dtype {features.dtype} != compute dtype {dt}")
        feat_mem, rpb, M_ext = _mem_geometry(features)
        vp = m.visual_projection
        mem = ops.linear(feat_mem, W(vp.weight, dt), vp.bias.detach())  # [M_ext, D]
        # key padding mask, uint8 [B,T] (converted once here, not per layer by attention_fwd)
        tgt_pad = (captions == m.pad_token_id).to(torch.uint8) if use_pad_mask else None
        # dropout (train mode, p = DecoderConfig.dropout): decoders.py:417 on the embeddings and,
        # per nn.TransformerDecoderLayer, MHA probabilities (self, cross), dropout1/2/3 on the
        # residual branches and the FFN inner dropout.  Masks are hashes of a per-site seed.
        p = m.dropout_p if m.training else 0.0
        seed = (lambda: (p, next_seed())) if p > 0 else (lambda: ops.NO_DROP)
        d_emb = seed()
        x = ops.embedding_fwd(captions, m.embedding.weight.detach(), m.position_encoding.weight.detach(), 0, dt,
                              drop=d_emb)
        BT = B * T
        saved_layers = []
        for L in m.transformer_decoder.layers:
            sa, ca = L.self_attn, L.multihead_attn
            drops = tuple(seed() for _ in range(6))  # sa-prob, dropout1, ca-prob, dropout2, ffn, dropout3
            x_in = x
            qkv = ops.linear(x, W(sa.in_proj_weight, dt), sa.in_proj_bias.detach())
            a = torch.empty(BT, D, dtype=dt, device=x.device)
            lse1, kp = ops.attention_fwd(heads(qkv, 0, B, T), heads(qkv, D, B, T), heads(qkv, 2 * D, B, T),
                                         heads(a, 0, B, T), B, H, T, T, hd, scale, causal=True, key_pad=tgt_pad,
                                         drop=drops[0])
            s1 = ops.linear(a, W(sa.out_proj.weight, dt), sa.out_proj.bias.detach(), residual=x, drop=drops[1])
            x1, mu1, rs1 = ops.layernorm_fwd(s1, L.norm1.weight.detach(), L.norm1.bias.detach(), L.norm1.eps)
            wca = W(ca.in_proj_weight, dt)
            bca = ca.in_proj_bias.detach()
            qc = ops.linear(x1, wca[:D], bca[:D])
            kv = ops.linear(mem, wca[D:], bca[D:])  # [M_ext, 2D]
            c = torch.empty(BT, D, dtype=dt, device=x.device)
            kvh_k = HeadView(kv, 0, rpb * 2 * D, 2 * D)
            kvh_v = HeadView(kv, D, rpb * 2 * D, 2 * D)
            lse2, _ = ops.attention_fwd(heads(qc, 0, B, T), kvh_k, kvh_v, heads(c, 0, B, T), B, H, T, S, hd, scale,
                                        drop=drops[2])
            s2 = ops.linear(c, W(ca.out_proj.weight, dt), ca.out_proj.bias.detach(), residual=x1, drop=drops[3])
            x2, mu2, rs2 = ops.layernorm_fwd(s2, L.norm2.weight.detach(), L.norm2.bias.detach(), L.norm2.eps)
            I = L.linear1.weight.shape[0]
            f_pre = torch.empty(BT, I, dtype=dt, device=x.device)
            f = ops.linear(x2, W(L.linear1.weight, dt), L.linear1.bias.detach(), act=ACT_GELU_ERF | ACT_DERIV, preact=f_pre,
                           drop=drops[4])
            s3 = ops.linear(f, W(L.linear2.weight, dt), L.linear2.bias.detach(), residual=x2, drop=drops[5])
            x, mu3, rs3 = ops.layernorm_fwd(s3, L.norm3.weight.detach(), L.norm3.bias.detach(), L.norm3.eps)
            saved_layers.append((x_in, qkv, a, lse1, kp, s1, mu1, rs1, x1, qc, kv, c, lse2, s2, mu2, rs2, x2, f_pre,
                                 f, s3, mu3, rs3, drops))
        ol = m.output_layer
        wout = ol.weight._capk_pad_bf16 if dt == torch.bfloat16 else ol.weight._capk_pad_master
        if dt == torch.bfloat16:
            # the LM head leaves the shifted CE's softmax partials (and where the CE backward may
            # write this head's bias gradient) on the logits buffer: capk/train/losses.py
            logits_pad, part = ops.linear_lse(x, wout, _pad_bias(ol), V)
            if part is not None:
                logits_pad._capk_ce_part = (part, logits_pad._version)
                logits_pad._capk_bias_grad = _pad_bias_grad(ol)
        else:
            logits_pad = ops.linear(x, wout, _pad_bias(ol))
        ctx.m = m
        ctx.d_emb = d_emb
        ctx.dims = (B, S, T, D, H, hd, scale, V, Vp, rpb, M_ext)
        ctx.saved = (feat_mem, mem, captions, saved_layers, x)
        ctx.features_meta = (features.shape, features.stride())
        logits = logits_pad[:, :V].view(B, T, V)
        hidden = x.view(B, T, D)
        ctx.logits_pad = logits_pad
        return logits, hidden

    @staticmethod
    def backward(ctx, dlogits, dhidden):
        m = ctx.m
        dt = m.cdtype
        B, S, T, D, H, hd, scale, V, Vp, rpb, M_ext = ctx.dims
        feat_mem, mem, captions, saved_layers, xT = ctx.saved
        ctx.saved = None
        BT = B * T
        dev = xT.device
        ol = m.output_layer
        # ---- LM head
        if dlogits is not None:
            dl = _padded_grad(dlogits, ctx.logits_pad, BT, V, Vp)
            ops.linear_dw(dl, xT, ol.weight._capk_pad_grad)
            if not getattr(dl, "_capk_bias_done", False):  # (else written by the CE backward's pass)
                ops.colsum(dl, _pad_bias_grad(ol))
            wout = ol.weight._capk_pad_bf16 if dt == torch.bfloat16 else ol.weight._capk_pad_master
            dx = ops.linear_dx(dl, wout)
        else:
            dx = torch.zeros(BT, D, dtype=dt, device=dev)
            ops.zero_(ol.weight._capk_pad_grad)
            ops.zero_(_pad_bias_grad(ol))
        if dhidden is not None:
            dx = dx + dhidden.reshape(BT, D)
        ctx.logits_pad = None
        store = store_of(m)
        notify_final(store, [ol.weight, ol.bias])  # (its bias gradient: here or by the CE backward)
        dmem = torch.empty(M_ext, D, dtype=dt, device=dev)
        first = True
        for li in range(len(saved_layers) - 1, -1, -1):
            L = m.transformer_decoder.layers[li]
            # the layer's LayerNorm / bias partial-sum finishes as one launch (ops.deferred_finishes)
            with ops.deferred_finishes():
                sa, ca = L.self_attn, L.multihead_attn
                (x_in, qkv, a, lse1, kp, s1, mu1, rs1, x1, qc, kv, c, lse2, s2, mu2, rs2, x2, f_pre, f, s3, mu3,
                 rs3, drops) = saved_layers[li]
                saved_layers[li] = None
                on = drops[1][0] > 0

                def ln_bwd(dy, s, norm, mu, rs, drop):
                    """grad of s = x + dropout(branch) through norm: (ds, ds * mask)."""
                    if not on:
                        g = ops.layernorm_bwd(dy, s, norm.weight.detach(), mu, rs, G(norm.weight), G(norm.bias))
                        return g, g
                    gm = torch.empty_like(s)
                    g = ops.layernorm_bwd(dy, s, norm.weight.detach(), mu, rs, G(norm.weight), G(norm.bias), drop=drop,
                                          out_drop=gm)
                    return g, gm

                # norm3(x2 + dropout3(linear2(dropout(gelu(linear1(x2))))))
                ds3, ds3m = ln_bwd(dx, s3, L.norm3, mu3, rs3, drops[5])
                dfp = linear_bwd(ds3m, f, L.linear2.weight, L.linear2.bias, dt, act_bwd=ACT_GELU_ERF | ACT_DERIV, aux=f_pre,
                                 drop=drops[4])
                ops.linear_dw(dfp, x2, G(L.linear1.weight))
                ops.colsum(dfp, G(L.linear1.bias))
                ops.linear_dx(dfp, W(L.linear1.weight, dt), out=ds3, beta=1.0)  # dx2 = ds3 + dfp W1
                # norm2(x1 + dropout2(MHA(x1, mem)))
                ds2, ds2m = ln_bwd(ds3, s2, L.norm2, mu2, rs2, drops[3])
                dc = linear_bwd(ds2m, c, ca.out_proj.weight, ca.out_proj.bias, dt)
                dqc = torch.empty(BT, D, dtype=dt, device=dev)
                dkv = torch.empty(M_ext, 2 * D, dtype=dt, device=dev)
                if rpb != S:
                    ops.zero_gap_rows(dkv, B, rpb, S)  # gap rows (e.g. ViT CLS rows) get no K/V gradient
                ops.attention_bwd(heads(qc, 0, B, T), HeadView(kv, 0, rpb * 2 * D, 2 * D),
                                  HeadView(kv, D, rpb * 2 * D, 2 * D), heads(c, 0, B, T), heads(dc, 0, B, T), lse2,
                                  heads(dqc, 0, B, T), HeadView(dkv, 0, rpb * 2 * D, 2 * D),
                                  HeadView(dkv, D, rpb * 2 * D, 2 * D), B, H, T, S, hd, scale, drop=drops[2])
                gW, gB = G(ca.in_proj_weight), G(ca.in_proj_bias)
                wca = W(ca.in_proj_weight, dt)
                ops.linear_dw(dkv, mem, gW[D:])
                ops.colsum(dkv, gB[D:])
                ops.linear_dx(dkv, wca[D:], out=dmem, beta=0.0 if first else 1.0)
                first = False
                ops.linear_dw(dqc, x1, gW[:D])
                ops.colsum(dqc, gB[:D])
                ops.linear_dx(dqc, wca[:D], out=ds2, beta=1.0)  # dx1 = ds2 + dqc Wq
                # norm1(x + dropout1(SA(x)))
                ds1, ds1m = ln_bwd(ds2, s1, L.norm1, mu1, rs1, drops[1])
                da = linear_bwd(ds1m, a, sa.out_proj.weight, sa.out_proj.bias, dt)
                dqkv = torch.empty_like(qkv)
                ops.attention_bwd(heads(qkv, 0, B, T), heads(qkv, D, B, T), heads(qkv, 2 * D, B, T), heads(a, 0, B, T),
                                  heads(da, 0, B, T), lse1, heads(dqkv, 0, B, T), heads(dqkv, D, B, T),
                                  heads(dqkv, 2 * D, B, T), B, H, T, T, hd, scale, causal=True, key_pad_u8=kp,
                                  drop=drops[0])
                ops.linear_dw(dqkv, x_in, G(sa.in_proj_weight))
                ops.colsum(dqkv, G(sa.in_proj_bias))
                ops.linear_dx(dqkv, W(sa.in_proj_weight, dt), out=ds1, beta=1.0)  # dx = ds1 + dqkv Win
                dx = ds1
            notify_final(store, L.parameters())  # this layer's gradients are complete
        # embeddings (scatter-add into zeroed grads; padding_idx rows skipped)
        ops.zero_(G(m.embedding.weight))
        ops.zero_(G(m.position_encoding.weight))
        ops.embedding_bwd(captions, dx, m.pad_token_id, G(m.embedding.weight), G(m.position_encoding.weight), 0,
                          drop=ctx.d_emb)
        notify_final(store, [m.embedding.weight, m.position_encoding.weight])
        # visual projection
        vp = m.visual_projection
        # gap rows of dmem are exactly zero: every dkv gap row is zero (see above)
        ops.linear_dw(dmem, feat_mem, G(vp.weight))
        ops.colsum(dmem, G(vp.bias))
        notify_final(store, [vp.weight, vp.bias])
        dfeat_mem = ops.linear_dx(dmem, W(vp.weight, dt))
        shape, stride = ctx.features_meta
        dfeatures = dfeat_mem.as_strided(shape, stride, 0)
        return dfeatures, None, None, None, None


def _pad_bias(ol):
    return ol.bias._capk_pad_master


def _pad_bias_grad(ol):
    return ol.bias._capk_pad_grad


def _padded_grad(dlogits, logits_pad, BT, V, Vp):
    """The CE kernel writes its gradient into a padded [BT, Vp] buffer and hands back a
    [B,T,V] view of it; recover that buffer (or pad a foreign gradient)."""
    base = dlogits._base
    if (base is not None and tuple(base.shape) == (BT, Vp) and base.data_ptr() == dlogits.data_ptr()
            and base.is_contiguous()):
        return base
    out = torch.zeros(BT, Vp, dtype=logits_pad.dtype, device=logits_pad.device)
    out[:, :V].copy_(dlogits.reshape(BT, V))
    return out


def _history_tables(R, L, dev):
    """Beam-history tables [R, L8] int32 (L rounded up to 8 for the 16-B row gather): the live
    table, a gather target, and the identity (row r holds every position of hypothesis r)."""
    L8 = (L + 7) // 8 * 8
    hist0 = torch.arange(R, dtype=torch.int32, device=dev)[:, None].expand(R, L8).contiguous()
    return hist0.clone(), torch.empty_like(hist0), hist0


def _history_reorder(hist, tmp, idx, t):
    """hist[r, :t] <- hist[idx[r], :t]; columns >= t keep row r (position t is written by row r's
    own step; position t-1 of the parent is the parent's own row, carried by the copy)."""
    R, L8 = hist.shape
    f = hist.view(torch.float32)  # bit copy through the fp32 row gather
    ops.check(ops.lib().capk_gather_rows(ops.dtype_code(f), 1, R, L8, idx.data_ptr(), f.data_ptr(), L8, 0,
                                         tmp.data_ptr(), L8, 0, ops._stream()), "capk_gather_rows")
    hist[:, :t].copy_(tmp[:, :t])


class KVDecodeRunner:
    """KV-cached incremental decode of the Transformer decoder for beam search
    (SURVEY §8a A14 on the A4 model; HF's per-step ``past_key_values`` path).

    Same arithmetic per position as the teacher-forced pass (eval mode, no pad mask,
    as ``generate`` runs it, decoders.py:473-477), one new token per beam per step:

    * memory side, once per image: visual projection and every layer's cross K/V
      ``[B*(S+gap), 2D]`` — the k beams of image b share them (the cross-attention runs
      with the k beam queries of image b as one batch entry: Nq = k);
    * self side: the fused QKV GEMM of the new token writes straight into the layer's
      cache slot ``cache[l, r, t, :]`` (layout [layers, B*k, max_length, 3D]); the
      attention reads keys/values 0..t of row r in place;
    * HF ``Cache.reorder_cache(beam_idx)`` (utils.py:3479-3489) without moving the cache: a
      beam-history table ``hist[r, j]`` (int32, the cache row holding position j of
      hypothesis r) is gathered by the step's parent indices (a few KB per step) and the
      self-attention reads key j < t from row ``hist[r, j]`` (capk_attention_decode_rows);
      the cache rows themselves are written once, by the QKV GEMM of their own step.  The
      former whole-cache gather (R x t x 3D per layer per step, ping-pong buffers) remains
      behind CAPK_KV_GATHER=1 for A/B and the bit-identity test.
    """

    def __init__(self, m, features, num_beams, max_length):
        dt = m.cdtype
        self.m, self.dt, self.k, self.Lmax = m, dt, num_beams, max_length
        B, S, D = features.shape
        self.B, self.S, self.D = B, S, D
        self.H = m.num_heads
        self.hd = D // self.H
        self.scale = 1.0 / math.sqrt(self.hd)
        feat_mem, self.rpb, _ = _mem_geometry(features)
        nl = len(m.transformer_decoder.layers)
        dev = features.device
        self.mem_kv = [torch.empty(feat_mem.shape[0], 2 * D, dtype=dt, device=dev) for _ in range(nl)]
        R = B * num_beams
        self.R = R
        shape = (nl, R, max_length, 3 * D)
        self.gather_kv = os.environ.get("CAPK_KV_GATHER", "0") == "1"
        self._bufs = (torch.empty(shape, dtype=dt, device=dev),
                      torch.empty(shape, dtype=dt, device=dev) if self.gather_kv else None)
        self.hist, self.hist_tmp, self.hist0 = _history_tables(R, max_length, dev)
        ol = m.output_layer
        self.wout = ol.weight._capk_pad_bf16 if dt == torch.bfloat16 else ol.weight._capk_pad_master
        self.bout = _pad_bias(ol)
        self.load(features)

    def load(self, features):
        """Per-call state, written in place (a runner reused by capk.graphs keeps its
        buffers): the memory side -- visual projection and every layer's cross K/V."""
        m, dt, D = self.m, self.dt, self.D
        if features.dtype != dt:
            raise TypeError(f"capk TransformerDecoder: features dtype {features.dtype} != compute dtype {dt}")
        feat_mem, rpb, _ = _mem_geometry(features)
        if tuple(features.shape) != (self.B, self.S, D) or rpb != self.rpb:
            raise ValueError("capk KVDecodeRunner.load: feature geometry differs from the runner's")
        vp = m.visual_projection
        mem = ops.linear(feat_mem, W(vp.weight, dt), vp.bias.detach())
        for li, L in enumerate(m.transformer_decoder.layers):
            ca = L.multihead_attn
            ops.linear(mem, W(ca.in_proj_weight, dt)[D:], ca.in_proj_bias.detach()[D:], out=self.mem_kv[li])
        self.reset()

    def reset(self):
        self.cache, self.spare = self._bufs
        self.hist.copy_(self.hist0)

    def reorder(self, idx, t):
        """Rows r <- idx[r] for cache positions [0, t): the history table (default), or every
        layer's cache in one gather launch (CAPK_KV_GATHER=1)."""
        if t <= 0:
            return
        if not self.gather_kv:
            _history_reorder(self.hist, self.hist_tmp, idx, t)
            return
        c = self.cache
        nl, R, Lm, C3 = c.shape
        check = ops.check
        check(ops.lib().capk_gather_rows(ops.dtype_code(c), nl, R, t * C3, idx.data_ptr(), c.data_ptr(), Lm * C3,
                                         R * Lm * C3, self.spare.data_ptr(), Lm * C3, R * Lm * C3, ops._stream()),
              "capk_gather_rows")
        self.cache, self.spare = self.spare, self.cache

    def step(self, cur_len, ids, reorder_idx):
        """Feed the tokens at position t = cur_len-1 for all B*k rows -> logits [R, Vp]."""
        m, dt, D, H, hd, R, k = self.m, self.dt, self.D, self.H, self.hd, self.R, self.k
        t = cur_len - 1
        if reorder_idx is not None:
            self.reorder(reorder_idx, t)
        Lm = self.Lmax
        x = ops.embedding_fwd(ids.view(R, 1), m.embedding.weight.detach(), m.position_encoding.weight.detach(), t, dt)
        rs_cache = Lm * 3 * D
        for li, L in enumerate(m.transformer_decoder.layers):
            sa, ca = L.self_attn, L.multihead_attn
            cl = self.cache[li]                      # [R, Lm, 3D]
            ops.linear(x, W(sa.in_proj_weight, dt), sa.in_proj_bias.detach(), out=cl[:, t, :])
            a = torch.empty(R, D, dtype=dt, device=x.device)
            qv, kv_, vv = (HeadView(cl, t * 3 * D, rs_cache, 3 * D), HeadView(cl, D, rs_cache, 3 * D),
                           HeadView(cl, 2 * D, rs_cache, 3 * D))
            if self.gather_kv:
                ops.attention_fwd(qv, kv_, vv, HeadView(a, 0, D, D), R, H, 1, t + 1, hd, self.scale)
            else:
                ops.attention_decode_rows(qv, kv_, vv, HeadView(a, 0, D, D), self.hist, R, H, 1, t + 1, hd,
                                          self.scale)
            # post-LN: each sublayer's output projection is summed by its LayerNorm (ops.product_ln)
            x1, _ = ops.product_ln(a, W(sa.out_proj.weight, dt), False, sa.out_proj.bias.detach(), x,
                                   L.norm1.weight.detach(), L.norm1.bias.detach(), L.norm1.eps)
            qc = ops.linear(x1, W(ca.in_proj_weight, dt)[:D], ca.in_proj_bias.detach()[:D])
            c = torch.empty(R, D, dtype=dt, device=x.device)
            kv = self.mem_kv[li]
            ops.attention_fwd(HeadView(qc, 0, k * D, D), HeadView(kv, 0, self.rpb * 2 * D, 2 * D),
                              HeadView(kv, D, self.rpb * 2 * D, 2 * D), HeadView(c, 0, k * D, D), self.B, H, k,
                              self.S, hd, self.scale)
            x2, _ = ops.product_ln(c, W(ca.out_proj.weight, dt), False, ca.out_proj.bias.detach(), x1,
                                   L.norm2.weight.detach(), L.norm2.bias.detach(), L.norm2.eps)
            f = ops.linear(x2, W(L.linear1.weight, dt), L.linear1.bias.detach(), act=ACT_GELU_ERF)
            x, _ = ops.product_ln(f, W(L.linear2.weight, dt), False, L.linear2.bias.detach(), x2,
                                  L.norm3.weight.detach(), L.norm3.bias.detach(), L.norm3.eps)
        return ops.linear(x, self.wout, self.bout)
