"""Attention-mechanism plugin surface — mirrors src/models/attention.py (SURVEY §8a
rows A7-A10).

``build_attention(AttentionConfig)`` returns modules with the reference's parameter
names and initialisation (``query_proj``, ``key_proj``, ``energy``, ... all
``nn.Linear``).  Inside the LSTM decoder they run through a step protocol on libcapk
kernels so that everything that does not depend on the decode step (the key / value
projections of the image features) is computed once per image instead of once per
step (the reference recomputes it every step; the values are identical):

  hoist(feats)                         per-image work            -> H
  step_fwd(H, t, q, h_mem, c_mem, ...) one decode step
  step_bwd(H, t, dctx, ...)            its backward, accumulating key/value grads
  finish_bwd(H, Q)                     per-image backward        -> d features

``forward(query, key, value, key_padding_mask, **kw)`` keeps the reference's standalone
contract (query [B, D] or [B, Q, D], key-padding mask, AdaptiveAttention's memory_state /
cell_state, differentiable returned weights) via the same protocol, one step per query.
"""
import os

import torch
import torch.nn as nn

from .. import _lib as ops_act_lib
from .. import ops
from ..config import AttentionConfig, AttentionType
from .common import G, CapkModule, W

_SOFT_DEFER = os.environ.get("CAPK_SOFT_DEFER", "1") != "0"


class ops_act:  # activation codes of the GEMM epilogue / act_bwd
    TANH = ops_act_lib.ACT_TANH
    SIGMOID = ops_act_lib.ACT_SIGMOID


class AttentionMechanism(nn.Module):
    """attention.py:9-35."""

    def forward(self, query, key, value, key_padding_mask=None, **kwargs):
        raise NotImplementedError


class _Hoist:
    pass


def _compact(feats):
    """[B, S, D] rows as one contiguous block (ViT/CLIP features carry a CLS-row gap)."""
    if feats.is_contiguous():
        return feats
    B, S, D = feats.shape
    out = torch.empty(B, S, D, dtype=feats.dtype, device=feats.device)
    idx = torch.arange(S, dtype=torch.int32, device=feats.device)
    ops.gather_rows(feats, idx, out, B, S, D, feats.stride(1), feats.stride(0), D, S * D)
    return out


class SoftAttention(AttentionMechanism, CapkModule):
    """attention.py:38-118: e = energy(tanh(Wq q + Wk k)) / T, masked_fill(-1e9), softmax, ctx = w v."""

    def __init__(self, config: AttentionConfig):
        super().__init__()
        self.query_dim = self.key_dim = self.hidden_dim = config.hidden_dim
        self.query_proj = nn.Linear(self.query_dim, self.hidden_dim)
        self.key_proj = nn.Linear(self.key_dim, self.hidden_dim)
        self.energy = nn.Linear(self.hidden_dim, 1)
        self.temperature = config.temperature

    # ---------------------------------------------------------- step protocol
    def hoist(self, keys, values, key_pad, steps):
        dt = self.cdtype
        H = _Hoist()
        H.keys, H.values = _compact(keys), (_compact(values) if values is not keys else None)
        B, S, D = H.keys.shape
        H.B, H.S, H.D, H.key_pad = B, S, D, key_pad
        H.kp = ops.linear(H.keys.view(B * S, D), W(self.key_proj.weight, dt), self.key_proj.bias.detach())
        H.w = torch.empty(steps, B, S, dtype=torch.float32, device=keys.device)
        H.qp = torch.empty(steps, B, D, dtype=dt, device=keys.device)
        return H

    def _v(self, H):
        return H.values if H.values is not None else H.keys

    def step_fwd(self, H, t, q, h_mem, c_mem, ctx_out):
        dt = self.cdtype
        ops.linear(q, W(self.query_proj.weight, dt), self.query_proj.bias.detach(), out=H.qp[t])
        ops.soft_attn_fwd(H.qp[t], H.kp.view(H.B, H.S, H.D), self._v(H), self.energy.weight.detach().view(-1),
                          self.energy.bias.detach(), 1.0 / self.temperature, ctx_out, H.w[t], key_pad=H.key_pad)
        return H.w[t]

    def begin_bwd(self, H):
        B, S, D, dev = H.B, H.S, H.D, H.kp.device
        steps = H.qp.shape[0]
        # deferred key / value gradients (capk_soft_attn_kv_grad after the last step) unless
        # CAPK_SOFT_DEFER=0: the steps stash their energies' gradients and output gradients
        H.defer = _SOFT_DEFER
        alloc = torch.empty if H.defer else torch.zeros
        H.dkp = alloc(B, S, D, dtype=torch.float32, device=dev)
        H.dv = alloc(B, S, D, dtype=torch.float32, device=dev)
        if H.defer:
            H.de_all = torch.zeros(steps, B, S, dtype=torch.float32, device=dev)
            H.dctx_all = torch.zeros(steps, B, D, dtype=self.cdtype, device=dev)
        H.dwe = torch.zeros(B, D, dtype=torch.float32, device=dev)
        H.dbe = torch.zeros(B, dtype=torch.float32, device=dev)
        H.dqp = torch.empty_like(H.qp)

    def step_bwd(self, H, t, dctx, dq_out, dq_residual=None, dc_mem_out=None, dw=None, dh_mem_out=None):
        """Writes dq_out = d(query) (+ dq_residual).  Soft attention does not read the LSTM states.
        dw: optional gradient on the returned weights (fp32 [B, S])."""
        dt = self.cdtype
        if H.defer:
            ops.soft_attn_bwd_step(H.qp[t], H.kp.view(H.B, H.S, H.D), self._v(H),
                                   self.energy.weight.detach().view(-1), 1.0 / self.temperature, H.w[t], dctx,
                                   H.dqp[t], H.dwe, H.dbe, H.de_all[t], H.dctx_all[t], dw_in=dw)
        else:
            ops.soft_attn_bwd(H.qp[t], H.kp.view(H.B, H.S, H.D), self._v(H), self.energy.weight.detach().view(-1),
                              1.0 / self.temperature, H.w[t], dctx, H.dqp[t], H.dkp, H.dv, H.dwe, H.dbe, dw_in=dw)
        ops.gemm(H.dqp[t], True, W(self.query_proj.weight, dt), False, H.B, H.D, H.D, dq_out, lda=H.D,
                 ldb=H.D, ldc=dq_out.stride(0), residual=dq_residual,
                 ldr=dq_residual.stride(0) if dq_residual is not None else 0)
        return False  # no memory/cell-state gradient

    def finish_bwd(self, H, Q):
        """Q: [steps*B, D] queries of every step (t-major).  Returns (dkeys, dvalues or None)."""
        dt = self.cdtype
        B, S, D = H.B, H.S, H.D
        if H.defer:
            ops.soft_attn_kv_grad(H.qp, H.kp.view(B, S, D), self.energy.weight.detach().view(-1), H.de_all, H.w,
                                  H.dctx_all, H.dkp, H.dv)
        steps = H.qp.shape[0]
        dqp = H.dqp.view(steps * B, D)
        ops.linear_dw(dqp, Q, G(self.query_proj.weight))
        ops.colsum(dqp, G(self.query_proj.bias))
        ops.colsum(H.dwe, G(self.energy.weight).view(-1))
        ops.add_rows(H.dbe, G(self.energy.bias), 1, 1, 1, 0, 0, B, 1, 0, 0, False)
        dkp = H.dkp.view(B * S, D)
        if dt != torch.float32:
            dkp_c = torch.empty(B * S, D, dtype=dt, device=dkp.device)
            ops.cast(dkp, dkp_c)
            dkp = dkp_c
        keys = H.keys.view(B * S, D)
        ops.linear_dw(dkp, keys, G(self.key_proj.weight))
        ops.colsum(dkp, G(self.key_proj.bias))
        dv = H.dv.view(B * S, D)
        if dt != torch.float32:
            dv_c = torch.empty(B * S, D, dtype=dt, device=dv.device)
            ops.cast(dv, dv_c)
            dv = dv_c
        if H.values is None:  # keys is values: one gradient
            dkeys = ops.linear_dx(dkp, W(self.key_proj.weight, dt), out=dv, beta=1.0)
            return dkeys.view(B, S, D), None
        return ops.linear_dx(dkp, W(self.key_proj.weight, dt)).view(B, S, D), dv.view(B, S, D)

    # ------------------------------------------------------------ standalone
    def forward(self, query, key, value, key_padding_mask=None, **kwargs):
        return _standalone(self, query, key, value, key_padding_mask, kwargs)


def _standalone(mod, query, key, value, key_padding_mask, kw):
    """AttentionMechanism.forward contract (attention.py:12-35): query [B, D] or [B, Q, D],
    key / value [B, S, D], key_padding_mask bool [B, S] (True = padding); returns
    (context [B, (Q,) D], weights [B, (Q,) S]).  The Q queries of an image run as Q steps of
    the hoisted step protocol (the key / value projections are computed once per call),
    which restates the reference's [B, Q, S, D] broadcast per query."""
    squeeze = query.dim() == 2
    q3 = query[:, None] if squeeze else query
    if q3.dim() != 3 or key.dim() != 3 or value.dim() != 3:
        raise ValueError("attention: query [B, D] | [B, Q, D], key / value [B, S, D]")
    h_mem, c_mem = kw.get("memory_state"), kw.get("cell_state")
    anchor = next(mod.parameters())
    ctx, w = _StandaloneFn.apply(q3, key, value, h_mem, c_mem, anchor, mod, key_padding_mask)
    if squeeze:
        return ctx[:, 0], w[:, 0]
    return ctx, w


class _StandaloneFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx_, q3, key, value, h_mem, c_mem, anchor, mod, key_padding_mask):
        dt = mod.cdtype
        B, Q, D = q3.shape
        kp = key_padding_mask.to(torch.uint8).contiguous() if key_padding_mask is not None else None
        same = key.data_ptr() == value.data_ptr() and key.stride() == value.stride() and key.shape == value.shape
        key_c = key.to(dt)
        val_c = key_c if same else value.to(dt)
        qt = q3.to(dt).transpose(0, 1).contiguous()  # step-major [Q, B, D]
        hm = h_mem.to(dt).contiguous() if h_mem is not None else None
        cm = c_mem.float().contiguous() if c_mem is not None else None
        H = mod.hoist(key_c, val_c, kp, Q)
        out = torch.empty(Q, B, D, dtype=dt, device=q3.device)
        for t in range(Q):
            mod.step_fwd(H, t, qt[t], hm, cm, out[t])
        w = H.w.transpose(0, 1).contiguous()  # [B, Q, S]
        ctx_.mod, ctx_.H, ctx_.qt, ctx_.same, ctx_.hm, ctx_.cm = mod, H, qt, same, hm, cm
        ctx_.in_dtypes = (q3.dtype, key.dtype, value.dtype,
                          h_mem.dtype if h_mem is not None else None, c_mem.dtype if c_mem is not None else None)
        return out.transpose(0, 1).to(q3.dtype), w

    @staticmethod
    def backward(ctx_, dout, dw):
        mod, H, qt = ctx_.mod, ctx_.H, ctx_.qt
        dt = mod.cdtype
        Q, B, D = qt.shape
        mod.begin_bwd(H)
        dq = torch.empty(Q, B, D, dtype=dt, device=qt.device)
        dh = torch.zeros(B, D, dtype=dt, device=qt.device) if ctx_.hm is not None else None
        dc = torch.zeros(B, D, dtype=torch.float32, device=qt.device) if ctx_.cm is not None else None
        dout_t = dout.to(dt).transpose(0, 1).contiguous() if dout is not None else torch.zeros_like(qt)
        dw_t = dw.float().transpose(0, 1).contiguous() if dw is not None else None
        for t in range(Q):
            mod.step_bwd(H, t, dout_t[t], dq[t], dc_mem_out=dc, dh_mem_out=dh,
                         dw=dw_t[t] if dw_t is not None else None)
        dk, dv = mod.finish_bwd(H, qt.view(Q * B, D))
        qd, kd, vd, hd_, cd = ctx_.in_dtypes
        dq3 = dq.transpose(0, 1).to(qd)
        dh = dh.to(hd_) if dh is not None else None
        dc = dc.to(cd) if dc is not None else None
        if ctx_.same:
            return dq3, dk.to(kd), None, dh, dc, None, None, None
        return dq3, dk.to(kd), dv.to(vd), dh, dc, None, None, None


class MultiHeadAttention(AttentionMechanism, CapkModule):
    """attention.py:121-218: q/k/v/o projections, softmax(q k^T / (T sqrt(hd))),
    masked_fill(-1e9) (the fused kernel uses -inf: identical unless every key of an image
    is padded), returned weights = mean over heads."""

    def __init__(self, config: AttentionConfig):
        super().__init__()
        self.num_heads = config.num_heads
        self.hidden_dim = config.hidden_dim
        assert self.hidden_dim % self.num_heads == 0, "Hidden dim must be divisible by num heads"
        self.head_dim = self.hidden_dim // self.num_heads
        self.temperature = config.temperature
        self.query_proj = nn.Linear(self.hidden_dim, self.hidden_dim)
        self.key_proj = nn.Linear(self.hidden_dim, self.hidden_dim)
        self.value_proj = nn.Linear(self.hidden_dim, self.hidden_dim)
        self.output_proj = nn.Linear(self.hidden_dim, self.hidden_dim)

    def hoist(self, keys, values, key_pad, steps):
        dt = self.cdtype
        H = _Hoist()
        H.keys = _compact(keys)
        H.values = _compact(values) if values is not keys else None
        B, S, D = H.keys.shape
        H.B, H.S, H.D, H.key_pad, H.kpu = B, S, D, key_pad, None
        dev = keys.device
        H.kh = ops.linear(H.keys.view(B * S, D), W(self.key_proj.weight, dt), self.key_proj.bias.detach())
        vals = (H.values if H.values is not None else H.keys).view(B * S, D)
        H.vh = ops.linear(vals, W(self.value_proj.weight, dt), self.value_proj.bias.detach())
        H.qh = torch.empty(steps, B, D, dtype=dt, device=dev)
        H.o = torch.empty(steps, B, D, dtype=dt, device=dev)
        H.w = torch.empty(steps, B, S, dtype=torch.float32, device=dev)
        H.lse = [None] * steps
        H.scale = 1.0 / (self.temperature * self.head_dim ** 0.5)
        return H

    def _views(self, H, t):
        B, S, D = H.B, H.S, H.D
        return (ops.HeadView(H.qh[t], 0, D, D), ops.HeadView(H.kh, 0, S * D, D), ops.HeadView(H.vh, 0, S * D, D),
                ops.HeadView(H.o[t], 0, D, D))

    def step_fwd(self, H, t, q, h_mem, c_mem, ctx_out):
        dt = self.cdtype
        ops.linear(q, W(self.query_proj.weight, dt), self.query_proj.bias.detach(), out=H.qh[t])
        qv, kv, vv, ov = self._views(H, t)
        H.lse[t], H.kpu = ops.attention_fwd(qv, kv, vv, ov, H.B, self.num_heads, 1, H.S, self.head_dim, H.scale,
                                            key_pad=H.key_pad)
        ops.attention_probs_mean(qv, kv, H.lse[t], H.B, self.num_heads, 1, H.S, self.head_dim, H.scale, H.w[t],
                                 key_pad=H.kpu)
        ops.linear(H.o[t], W(self.output_proj.weight, dt), self.output_proj.bias.detach(), out=ctx_out)
        return H.w[t]

    def begin_bwd(self, H):
        B, S, D, dev, dt = H.B, H.S, H.D, H.kh.device, self.cdtype
        H.dK = torch.zeros(B * S, D, dtype=torch.float32, device=dev)
        H.dV = torch.zeros(B * S, D, dtype=torch.float32, device=dev)
        H.sk = torch.empty(B * S, D, dtype=dt, device=dev)
        H.sv = torch.empty(B * S, D, dtype=dt, device=dev)
        H.dqh = torch.empty_like(H.qh)
        H.dctx = torch.empty_like(H.o)
        H.do = torch.empty(B, D, dtype=dt, device=dev)

    def step_bwd(self, H, t, dctx, dq_out, dq_residual=None, dc_mem_out=None, dw=None, dh_mem_out=None):
        """dw: optional gradient on the returned head-mean weights (fp32 [B, S])."""
        dt = self.cdtype
        B, S, D = H.B, H.S, H.D
        ops.copy_rows(dctx, H.dctx[t])
        ops.linear_dx(dctx, W(self.output_proj.weight, dt), out=H.do)
        qv, kv, vv, ov = self._views(H, t)
        ops.attention_bwd(qv, kv, vv, ov, ops.HeadView(H.do, 0, D, D), H.lse[t], ops.HeadView(H.dqh[t], 0, D, D),
                          ops.HeadView(H.sk, 0, S * D, D), ops.HeadView(H.sv, 0, S * D, D), B, self.num_heads, 1, S,
                          self.head_dim, H.scale, key_pad_u8=H.kpu)
        if dw is not None:  # attention.py:211 weights.mean(dim=1) is differentiable
            ops.attention_probs_mean_bwd(qv, kv, H.lse[t], dw, ops.HeadView(H.dqh[t], 0, D, D),
                                         ops.HeadView(H.dK, 0, S * D, D), B, self.num_heads, 1, S, self.head_dim,
                                         H.scale, key_pad=H.kpu)
        ops.add_rows(H.sk, H.dK, 1, B * S, D, 0, D, 1, 0, 0, D, True)
        ops.add_rows(H.sv, H.dV, 1, B * S, D, 0, D, 1, 0, 0, D, True)
        ops.gemm(H.dqh[t], True, W(self.query_proj.weight, dt), False, B, D, D, dq_out, lda=D, ldb=D,
                 ldc=dq_out.stride(0), residual=dq_residual,
                 ldr=dq_residual.stride(0) if dq_residual is not None else 0)
        return False

    def finish_bwd(self, H, Q):
        dt = self.cdtype
        B, S, D = H.B, H.S, H.D
        steps = H.qh.shape[0]
        dctx = H.dctx.view(steps * B, D)
        ops.linear_dw(dctx, H.o.view(steps * B, D), G(self.output_proj.weight))
        ops.colsum(dctx, G(self.output_proj.bias))
        dqh = H.dqh.view(steps * B, D)
        ops.linear_dw(dqh, Q, G(self.query_proj.weight))
        ops.colsum(dqh, G(self.query_proj.bias))
        outs = []
        for acc, proj, x in ((H.dK, self.key_proj, H.keys), (H.dV, self.value_proj,
                                                              H.values if H.values is not None else H.keys)):
            g = acc
            if dt != torch.float32:
                g = torch.empty(B * S, D, dtype=dt, device=acc.device)
                ops.cast(acc, g)
            ops.linear_dw(g, x.view(B * S, D), G(proj.weight))
            ops.colsum(g, G(proj.bias))
            outs.append(g)
        dkeys = ops.linear_dx(outs[0], W(self.key_proj.weight, dt))
        if H.values is None:
            ops.linear_dx(outs[1], W(self.value_proj.weight, dt), out=dkeys, beta=1.0)
            return dkeys.view(B, S, D), None
        return dkeys.view(B, S, D), ops.linear_dx(outs[1], W(self.value_proj.weight, dt)).view(B, S, D)

    def forward(self, query, key, value, key_padding_mask=None, **kwargs):
        return _standalone(self, query, key, value, key_padding_mask, kwargs)


class AdaptiveAttention(AttentionMechanism, CapkModule):
    """attention.py:221-294: visual sentinel s = W_p(sigmoid(W_s [q; h]) * tanh(c)),
    base attention ctx, beta = sigmoid(W_a [ctx; s]), out = beta ctx + (1 - beta) s."""

    def __init__(self, config: AttentionConfig):
        super().__init__()
        self.hidden_dim = config.hidden_dim
        self.base_attention = MultiHeadAttention(config) if config.num_heads > 1 else SoftAttention(config)
        self.sentinel_gate = nn.Linear(self.hidden_dim * 2, self.hidden_dim)
        self.sentinel_proj = nn.Linear(self.hidden_dim, self.hidden_dim)
        self.adaptive_weight = nn.Linear(self.hidden_dim * 2, 1)

    def hoist(self, keys, values, key_pad, steps):
        dt = self.cdtype
        H = _Hoist()
        H.base = self.base_attention.hoist(keys, values, key_pad, steps)
        B, D, dev = H.base.B, H.base.D, keys.device
        H.B, H.D = B, D
        H.cat1 = torch.empty(steps, B, 2 * D, dtype=dt, device=dev)
        H.sgpre = torch.empty(steps, B, D, dtype=dt, device=dev)
        H.sg = torch.empty(steps, B, D, dtype=dt, device=dev)
        H.sin = torch.empty(steps, B, D, dtype=dt, device=dev)
        H.cat2 = torch.empty(steps, B, 2 * D, dtype=dt, device=dev)
        H.beta = torch.empty(steps, B, dtype=torch.float32, device=dev)
        H.c = [None] * steps
        return H

    def step_fwd(self, H, t, q, h_mem, c_mem, ctx_out):
        dt = self.cdtype
        D = H.D
        ops.copy_rows(q, H.cat1[t][:, :D])
        ops.copy_rows(h_mem, H.cat1[t][:, D:])
        ops.linear(H.cat1[t], W(self.sentinel_gate.weight, dt), self.sentinel_gate.bias.detach(),
                   act=ops_act.SIGMOID, preact=H.sgpre[t], out=H.sg[t])
        ops.tanh_gate_fwd(c_mem, H.sg[t], H.sin[t])
        ops.linear(H.sin[t], W(self.sentinel_proj.weight, dt), self.sentinel_proj.bias.detach(), out=H.cat2[t][:, D:])
        w = self.base_attention.step_fwd(H.base, t, q, h_mem, c_mem, H.cat2[t][:, :D])
        ops.gate_mix_fwd(H.cat2[t][:, :D], H.cat2[t][:, D:], self.adaptive_weight.weight.detach().view(-1),
                         self.adaptive_weight.bias.detach(), H.beta[t], ctx_out)
        H.c[t] = c_mem
        H.w = H.base.w
        return w

    def begin_bwd(self, H):
        dt, B, D, dev = self.cdtype, H.B, H.D, H.cat1.device
        self.base_attention.begin_bwd(H.base)
        steps = H.cat1.shape[0]
        H.dwa = torch.zeros(2 * D, dtype=torch.float32, device=dev)
        H.dba = torch.zeros(1, dtype=torch.float32, device=dev)
        H.dctxb = torch.empty(B, D, dtype=dt, device=dev)
        H.dsp = torch.empty(steps, B, D, dtype=dt, device=dev)
        H.dsgpre = torch.empty(steps, B, D, dtype=dt, device=dev)
        H.dsg = torch.empty(B, D, dtype=dt, device=dev)

    def step_bwd(self, H, t, dctx, dq_out, dq_residual=None, dc_mem_out=None, dw=None, dh_mem_out=None):
        """dc_mem_out (fp32) and dh_mem_out ACCUMULATE; without dh_mem_out the memory-state half
        of the sentinel gate goes to dq_out (the LSTM decoder passes h_top as both)."""
        dt = self.cdtype
        B, D = H.B, H.D
        ops.gate_mix_bwd(H.cat2[t][:, :D], H.cat2[t][:, D:], self.adaptive_weight.weight.detach().view(-1),
                         H.beta[t], dctx, H.dctxb, H.dsp[t], H.dwa, H.dba)
        dsin = ops.linear_dx(H.dsp[t], W(self.sentinel_proj.weight, dt))
        if dc_mem_out is None:
            raise RuntimeError("AdaptiveAttention needs the cell-state gradient buffer")
        ops.tanh_gate_bwd(H.c[t], H.sg[t], dsin, H.dsg, dc_mem_out)
        ops.act_bwd(H.dsg, H.sgpre[t], ops_act.SIGMOID, out=H.dsgpre[t])
        self.base_attention.step_bwd(H.base, t, H.dctxb, dq_out, dq_residual, dw=dw)
        wsg = W(self.sentinel_gate.weight, dt)  # [D, 2D]: query half, memory-state half
        for half, dst in ((wsg[:, :D], dq_out), (wsg[:, D:], dq_out if dh_mem_out is None else dh_mem_out)):
            ops.gemm(H.dsgpre[t], True, half, False, B, D, D, dst, lda=D, ldb=2 * D, ldc=dst.stride(0), beta=1.0)
        return True

    def finish_bwd(self, H, Q):
        B, D = H.B, H.D
        steps = H.cat1.shape[0]
        g = H.dsgpre.view(steps * B, D)
        ops.linear_dw(g, H.cat1.view(steps * B, 2 * D), G(self.sentinel_gate.weight))
        ops.colsum(g, G(self.sentinel_gate.bias))
        g = H.dsp.view(steps * B, D)
        ops.linear_dw(g, H.sin.view(steps * B, D), G(self.sentinel_proj.weight))
        ops.colsum(g, G(self.sentinel_proj.bias))
        ops.copy_rows(H.dwa.view(1, 2 * D), G(self.adaptive_weight.weight))
        ops.add_rows(H.dba, G(self.adaptive_weight.bias), 1, 1, 1, 0, 0, 1, 1, 0, 0, False)
        return self.base_attention.finish_bwd(H.base, Q)

    def forward(self, query, key, value, key_padding_mask=None, memory_state=None, cell_state=None, **kwargs):
        """attention.py:242-294; memory_state / cell_state [B, D] are shared by the Q queries."""
        assert memory_state is not None and cell_state is not None, \
            "AdaptiveAttention requires memory_state and cell_state"
        return _standalone(self, query, key, value, key_padding_mask,
                           dict(kwargs, memory_state=memory_state, cell_state=cell_state))


class AttentionOnAttention(AttentionMechanism, CapkModule):
    """attention.py:297-360: ctx = base(q, k, v); cat = [ctx; W_q q];
    out = tanh(W_i cat + b_i) * sigmoid(W_g cat + b_g)."""

    def __init__(self, config: AttentionConfig):
        super().__init__()
        self.hidden_dim = config.hidden_dim
        self.base_attention = MultiHeadAttention(config) if config.num_heads > 1 else SoftAttention(config)
        self.query_proj = nn.Linear(self.hidden_dim, self.hidden_dim)
        self.info_vector_proj = nn.Sequential(nn.Linear(self.hidden_dim * 2, self.hidden_dim), nn.Tanh())
        self.info_gate_proj = nn.Sequential(nn.Linear(self.hidden_dim * 2, self.hidden_dim), nn.Sigmoid())

    def hoist(self, keys, values, key_pad, steps):
        dt = self.cdtype
        H = _Hoist()
        H.base = self.base_attention.hoist(keys, values, key_pad, steps)
        B, D, dev = H.base.B, H.base.D, keys.device
        H.B, H.D = B, D
        mk = lambda n: torch.empty(steps, B, n, dtype=dt, device=dev)  # noqa: E731
        H.cat, H.ipre, H.info, H.gpre, H.gate = mk(2 * D), mk(D), mk(D), mk(D), mk(D)
        return H

    def step_fwd(self, H, t, q, h_mem, c_mem, ctx_out):
        dt = self.cdtype
        D = H.D
        w = self.base_attention.step_fwd(H.base, t, q, h_mem, c_mem, H.cat[t][:, :D])
        ops.linear(q, W(self.query_proj.weight, dt), self.query_proj.bias.detach(), out=H.cat[t][:, D:])
        iv, ig = self.info_vector_proj[0], self.info_gate_proj[0]
        ops.linear(H.cat[t], W(iv.weight, dt), iv.bias.detach(), act=ops_act.TANH, preact=H.ipre[t], out=H.info[t])
        ops.linear(H.cat[t], W(ig.weight, dt), ig.bias.detach(), act=ops_act.SIGMOID, preact=H.gpre[t],
                   out=H.gate[t])
        ops.ew_mul(H.info[t], H.gate[t], ctx_out)
        H.w = H.base.w
        return w

    def begin_bwd(self, H):
        dt, B, D, dev = self.cdtype, H.B, H.D, H.cat.device
        self.base_attention.begin_bwd(H.base)
        steps = H.cat.shape[0]
        H.dipre = torch.empty(steps, B, D, dtype=dt, device=dev)
        H.dgpre = torch.empty(steps, B, D, dtype=dt, device=dev)
        H.dqa = torch.empty(steps, B, D, dtype=dt, device=dev)
        H.tmp = torch.empty(B, D, dtype=dt, device=dev)
        H.dcat = torch.empty(B, 2 * D, dtype=dt, device=dev)

    def step_bwd(self, H, t, dctx, dq_out, dq_residual=None, dc_mem_out=None, dw=None, dh_mem_out=None):
        dt = self.cdtype
        B, D = H.B, H.D
        iv, ig = self.info_vector_proj[0], self.info_gate_proj[0]
        ops.ew_mul(dctx, H.gate[t], H.tmp)
        ops.act_bwd(H.tmp, H.ipre[t], ops_act.TANH, out=H.dipre[t])
        ops.ew_mul(dctx, H.info[t], H.tmp)
        ops.act_bwd(H.tmp, H.gpre[t], ops_act.SIGMOID, out=H.dgpre[t])
        ops.linear_dx(H.dipre[t], W(iv.weight, dt), out=H.dcat)
        ops.linear_dx(H.dgpre[t], W(ig.weight, dt), out=H.dcat, beta=1.0)
        ops.copy_rows(H.dcat[:, D:], H.dqa[t])
        self.base_attention.step_bwd(H.base, t, H.dcat[:, :D], dq_out, dq_residual, dw=dw)
        ops.gemm(H.dqa[t], True, W(self.query_proj.weight, dt), False, B, D, D, dq_out, lda=D, ldb=D,
                 ldc=dq_out.stride(0), beta=1.0)
        return False

    def finish_bwd(self, H, Q):
        B, D = H.B, H.D
        steps = H.cat.shape[0]
        cat = H.cat.view(steps * B, 2 * D)
        for g, lin in ((H.dipre, self.info_vector_proj[0]), (H.dgpre, self.info_gate_proj[0])):
            g = g.view(steps * B, D)
            ops.linear_dw(g, cat, G(lin.weight))
            ops.colsum(g, G(lin.bias))
        g = H.dqa.view(steps * B, D)
        ops.linear_dw(g, Q, G(self.query_proj.weight))
        ops.colsum(g, G(self.query_proj.bias))
        return self.base_attention.finish_bwd(H.base, Q)

    def forward(self, query, key, value, key_padding_mask=None, **kwargs):
        return _standalone(self, query, key, value, key_padding_mask, kwargs)


def build_attention(config: AttentionConfig) -> AttentionMechanism:
    """attention.py:363-376 (D2: string types accepted)."""
    at = config.attention_type if isinstance(config.attention_type, AttentionType) else \
        AttentionType(config.attention_type)
    if at == AttentionType.SOFT:
        return SoftAttention(config)
    if at == AttentionType.MULTI_HEAD:
        return MultiHeadAttention(config)
    if at == AttentionType.ADAPTIVE:
        return AdaptiveAttention(config)
    if at == AttentionType.AOA:
        return AttentionOnAttention(config)
    raise ValueError(f"Unsupported attention type: {config.attention_type}")
