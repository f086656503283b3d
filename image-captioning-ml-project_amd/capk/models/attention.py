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

``forward(query, key, value, key_padding_mask)`` keeps the reference's standalone
contract (one query per image) via the same protocol.
"""
import torch
import torch.nn as nn

from .. import ops
from ..config import AttentionConfig, AttentionType
from .common import G, CapkModule, W


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
        H.dkp = torch.zeros(B, S, D, dtype=torch.float32, device=dev)
        H.dv = torch.zeros(B, S, D, dtype=torch.float32, device=dev)
        H.dwe = torch.zeros(B, D, dtype=torch.float32, device=dev)
        H.dbe = torch.zeros(B, dtype=torch.float32, device=dev)
        H.dqp = torch.empty_like(H.qp)

    def step_bwd(self, H, t, dctx, dq_out, dq_residual=None, dc_mem_out=None):
        """Writes dq_out = d(query) (+ dq_residual).  Soft attention does not read the LSTM states."""
        dt = self.cdtype
        ops.soft_attn_bwd(H.qp[t], H.kp.view(H.B, H.S, H.D), self._v(H), self.energy.weight.detach().view(-1),
                          1.0 / self.temperature, H.w[t], dctx, H.dqp[t], H.dkp, H.dv, H.dwe, H.dbe)
        ops.gemm(H.dqp[t], True, W(self.query_proj.weight, dt), False, H.B, H.D, H.D, dq_out, lda=H.D,
                 ldb=H.D, ldc=dq_out.stride(0), residual=dq_residual,
                 ldr=dq_residual.stride(0) if dq_residual is not None else 0)
        return False  # no memory/cell-state gradient

    def finish_bwd(self, H, Q):
        """Q: [steps*B, D] queries of every step (t-major).  Returns (dkeys, dvalues or None)."""
        dt = self.cdtype
        B, S, D = H.B, H.S, H.D
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
    squeeze = query.dim() == 2
    q = query if squeeze else query.reshape(query.shape[0], -1)
    if not squeeze and query.shape[1] != 1:
        raise NotImplementedError("capk attention modules: one query per image (the LSTM decode step)")
    ctx, w = _StandaloneFn.apply(q.contiguous(), key, value, mod.query_proj.weight, mod, key_padding_mask,
                                 kw.get("memory_state"), kw.get("cell_state"))
    if not squeeze:
        return ctx[:, None], w[:, None]
    return ctx, w


class _StandaloneFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx_, q, key, value, anchor, mod, key_padding_mask, h_mem, c_mem):
        kp = key_padding_mask.to(torch.uint8).contiguous() if key_padding_mask is not None else None
        same = key.data_ptr() == value.data_ptr() and key.stride() == value.stride()
        H = mod.hoist(key, key if same else value, kp, 1)
        B, D = q.shape
        out = torch.empty(B, D, dtype=q.dtype, device=q.device)
        w = mod.step_fwd(H, 0, q, h_mem, c_mem, out)
        ctx_.mod, ctx_.H, ctx_.q, ctx_.same = mod, H, q, same
        ctx_.shapes = (key.shape, value.shape)
        return out, w.clone()

    @staticmethod
    def backward(ctx_, dout, dw):
        mod, H, q = ctx_.mod, ctx_.H, ctx_.q
        mod.begin_bwd(H)
        dq = torch.empty_like(q)
        mod.step_bwd(H, 0, dout.contiguous(), dq)
        dk, dv = mod.finish_bwd(H, q)
        if ctx_.same:
            return dq, dk, None, None, None, None, None, None
        return dq, dk, dv, None, None, None, None, None


class MultiHeadAttention(AttentionMechanism, CapkModule):
    """attention.py:121-218 (parameters; the LSTM step path is row A8)."""

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

    def hoist(self, *a, **k):
        raise NotImplementedError("capk: MultiHeadAttention inside the LSTM decoder (SURVEY A8) is next")

    def forward(self, query, key, value, key_padding_mask=None, **kwargs):
        raise NotImplementedError("capk: MultiHeadAttention module (SURVEY A8) is next")


class AdaptiveAttention(AttentionMechanism, CapkModule):
    """attention.py:221-294 (parameters; the step path is row A10)."""

    def __init__(self, config: AttentionConfig):
        super().__init__()
        self.hidden_dim = config.hidden_dim
        self.base_attention = MultiHeadAttention(config) if config.num_heads > 1 else SoftAttention(config)
        self.sentinel_gate = nn.Linear(self.hidden_dim * 2, self.hidden_dim)
        self.sentinel_proj = nn.Linear(self.hidden_dim, self.hidden_dim)
        self.adaptive_weight = nn.Linear(self.hidden_dim * 2, 1)

    def hoist(self, *a, **k):
        raise NotImplementedError("capk: AdaptiveAttention (SURVEY A10) is next")

    def forward(self, query, key, value, key_padding_mask=None, memory_state=None, cell_state=None, **kwargs):
        assert memory_state is not None and cell_state is not None, \
            "AdaptiveAttention requires memory_state and cell_state"
        raise NotImplementedError("capk: AdaptiveAttention (SURVEY A10) is next")


class AttentionOnAttention(AttentionMechanism, CapkModule):
    """attention.py:297-360 (parameters; the step path is row A9)."""

    def __init__(self, config: AttentionConfig):
        super().__init__()
        self.hidden_dim = config.hidden_dim
        self.base_attention = MultiHeadAttention(config) if config.num_heads > 1 else SoftAttention(config)
        self.query_proj = nn.Linear(self.hidden_dim, self.hidden_dim)
        self.info_vector_proj = nn.Sequential(nn.Linear(self.hidden_dim * 2, self.hidden_dim), nn.Tanh())
        self.info_gate_proj = nn.Sequential(nn.Linear(self.hidden_dim * 2, self.hidden_dim), nn.Sigmoid())

    def hoist(self, *a, **k):
        raise NotImplementedError("capk: AttentionOnAttention (SURVEY A9) is next")

    def forward(self, query, key, value, key_padding_mask=None, **kwargs):
        raise NotImplementedError("capk: AttentionOnAttention (SURVEY A9) is next")


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
