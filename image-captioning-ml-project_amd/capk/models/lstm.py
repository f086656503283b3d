"""LSTM caption decoder on libcapk kernels (with A7-A10 attention).

Restates src/models/decoders.py:70-314 (LSTMDecoder).  Parameter names match the
reference (``embedding``, ``lstm.weight_ih_l{k}`` / ``weight_hh_l{k}`` / ``bias_*``,
``attention.*``, ``output_layer``, ``init_h``, ``init_c``).

Teacher-forced pass = one autograd Function over the whole caption:
  * h0/c0 = init_h/init_c(pooled) (GEMMs; c kept fp32);
  * embeddings of all steps and their layer-0 input projection are ONE GEMM before the
    loop (x_t W_ih0[:, :E]^T); per step only the recurrent GEMMs remain:
      layer 0: gates = pre_t + ctx_{t-1} W_ih0[:, E:]^T + h W_hh0^T + b_hh0
      layer l: gates = h_{l-1}' W_ih_l^T + b_ih_l + h_l W_hh_l^T + b_hh_l
    then the fused cell kernel (fp32 cell state; inter-layer dropout on the copy that
    feeds the next layer);
  * attention step (query = top h, memory/cell = h[-1]/c[-1]) — key/value projections
    of the image features hoisted out of the loop;
  * logits = output_layer(dropout(ctx)) for all steps as ONE GEMM after the loop.
Backward runs the recurrence in reverse with per-step GEMMs for the state/input
gradients and batches every weight gradient into one GEMM over all steps.  Step
buffers are t-major ([T, B, ...]); the LM head works on b-major rows so the logits are
the [B, T, V] view the CE kernel consumes.
"""
import math
import os

import torch
import torch.nn as nn

from .. import ops
from .common import G, CapkModule, W, next_seed
from .transformer import _pad64, _pad_bias, _pad_bias_grad, _padded_grad
from .attention import build_attention

# bf16 teacher-forced pass: each step-and-layer recurrence as ONE two-segment product into
# fp32 split-K slabs that the cell kernel sums (capk_gemm_pair_slabs), instead of two GEMMs
# and two split-K reduces.  CAPK_LSTM_PAIR=0 restores the per-GEMM route (A/B).
_PAIR = os.environ.get("CAPK_LSTM_PAIR", "1") != "0"


class _LSTMParams(nn.Module):
    """nn.LSTM's parameters (names + uniform(-1/sqrt(H), 1/sqrt(H)) init) without its cuDNN state."""

    def __init__(self, input_size, hidden_size, num_layers):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        k = 1.0 / math.sqrt(hidden_size)
        for layer in range(num_layers):
            inp = input_size if layer == 0 else hidden_size
            for name, shape in ((f"weight_ih_l{layer}", (4 * hidden_size, inp)),
                                (f"weight_hh_l{layer}", (4 * hidden_size, hidden_size)),
                                (f"bias_ih_l{layer}", (4 * hidden_size,)), (f"bias_hh_l{layer}", (4 * hidden_size,))):
                p = nn.Parameter(torch.empty(shape))
                nn.init.uniform_(p, -k, k)
                self.register_parameter(name, p)

    def w(self, kind, layer):
        return getattr(self, f"{kind}_l{layer}")


class LSTMDecoderCore(CapkModule):
    def __init__(self, config, attention_config, vocab_size, pad_token_id, embedding_dim=None):
        super().__init__()
        self.hidden_dim = config.hidden_dim
        self.embedding_dim = embedding_dim or config.hidden_dim
        self.num_layers = config.num_layers
        self.vocab_size = vocab_size
        self.vocab_pad = _pad64(vocab_size)
        self.dropout_p = config.dropout
        self.pad_token_id = pad_token_id
        self.embedding = nn.Embedding(vocab_size, self.embedding_dim, padding_idx=pad_token_id)
        self.lstm = _LSTMParams(self.embedding_dim + self.hidden_dim, self.hidden_dim, self.num_layers)
        self.attention = build_attention(attention_config)
        self.output_layer = nn.Linear(self.hidden_dim, vocab_size)
        self.output_layer.weight._capk_pad_rows = self.vocab_pad
        self.output_layer.bias._capk_pad_rows = self.vocab_pad
        self.init_h = nn.Linear(self.hidden_dim, self.hidden_dim * self.num_layers)
        self.init_c = nn.Linear(self.hidden_dim, self.hidden_dim * self.num_layers)
        self.dropout = nn.Dropout(self.dropout_p)

    def forward_logits(self, features, pooled, captions):
        """-> (logits [B,T,V] view, attention_weights [B,T,S] view)."""
        return _LSTMFn.apply(features, pooled, captions, self.output_layer.weight, self)


class _LSTMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, features, pooled, captions, anchor, m):
        ctx.set_materialize_grads(False)
        dt = m.cdtype
        dev = captions.device
        B, T = captions.shape
        D, E, L = m.hidden_dim, m.embedding_dim, m.num_layers
        V, Vp = m.vocab_size, m.vocab_pad
        lstm, att = m.lstm, m.attention
        if features.dtype != dt or pooled.dtype != dt:
            raise TypeError(f"capk LSTMDecoder: feature dtype {features.dtype}/{pooled.dtype} != compute dtype {dt}")
        p = m.dropout_p if m.training else 0.0
        drop = (lambda: (p, next_seed())) if p > 0 else (lambda: ops.NO_DROP)
        pooled = pooled.contiguous()
        # initial states (decoders.py:122-135): layer l = columns [l*D, (l+1)*D)
        h0 = ops.linear(pooled, W(m.init_h.weight, dt), m.init_h.bias.detach())
        c0 = ops.linear(pooled, W(m.init_c.weight, dt), m.init_c.bias.detach(), out_dtype=torch.float32)
        Hs = [torch.empty(T + 1, B, D, dtype=dt, device=dev) for _ in range(L)]
        Cs = [torch.empty(T + 1, B, D, dtype=torch.float32, device=dev) for _ in range(L)]
        for layer in range(L):
            ops.copy_rows(h0[:, layer * D:(layer + 1) * D], Hs[layer][0])
            ops.copy_rows(c0[:, layer * D:(layer + 1) * D], Cs[layer][0])
        # embeddings, t-major rows (t*B + b), dropout (decoders.py:172-173)
        ids_t = captions.t().contiguous()
        d_emb = drop()
        emb = ops.embedding_fwd(ids_t, m.embedding.weight.detach(), None, 0, dt, drop=d_emb)  # [T*B, E]
        w_ih0 = W(lstm.weight_ih_l0, dt)
        pre0 = ops.linear(emb, w_ih0[:, :E], lstm.bias_ih_l0.detach())  # [T*B, 4D]
        CtxT = torch.zeros(T + 1, B, D, dtype=dt, device=dev)  # ctx_{t-1} feeds step t; row 0 = zeros
        H = att.hoist(features, features, None, T)
        acts = [torch.empty(T, B, 4 * D, dtype=dt, device=dev) for _ in range(L)]
        Hd = [torch.empty(T, B, D, dtype=dt, device=dev) for _ in range(L - 1)] if p > 0 else None
        drops = [[drop() for _ in range(L - 1)] for _ in range(T)]
        gates = torch.empty(B, 4 * D, dtype=dt, device=dev)
        pair = dt == torch.bfloat16 and _PAIR and D % 128 == 0  # (seams on 128-column tiles)
        if pair:
            # gates = [x | h] [W_ih | W_hh]^T (K seam at D) as fp32 slabs summed in the cell
            wsf = torch.empty(ops.pair_slabs_plan(B, 4 * D, 2 * D)[1], dtype=torch.float32, device=dev)
        for t in range(T):
            for layer in range(L):
                if pair:
                    if layer == 0:  # x = ctx_{t-1} against W_ih0[:, E:]; pre0 carries the embedding half + b_ih
                        a1, b1, ldb1, res, ba = CtxT[t], w_ih0[:, E:], E + D, pre0[t * B:(t + 1) * B], None
                    else:
                        a1 = Hd[layer - 1][t] if Hd is not None else Hs[layer - 1][t + 1]
                        b1, ldb1, res = W(lstm.w("weight_ih", layer), dt), D, None
                        ba = lstm.w("bias_ih", layer).detach()
                    sf = ops.gemm_pair_slabs(B, 4 * D, 2 * D, a1, D, b1, ldb1, True, wsf, A2=Hs[layer][t], lda2=D,
                                             B2=W(lstm.w("weight_hh", layer), dt), ldb2=D, k1=D)
                    hd = Hd[layer][t] if (Hd is not None and layer < L - 1) else None
                    ops.lstm_cell_fwd_slabs(wsf, sf, 4 * D, ba, lstm.w("bias_hh", layer).detach(), res, Cs[layer][t],
                                            Cs[layer][t + 1], Hs[layer][t + 1], acts[layer][t], h_drop=hd,
                                            drop=drops[t][layer] if hd is not None else ops.NO_DROP)
                    continue
                if layer == 0:
                    ops.gemm(CtxT[t], True, w_ih0[:, E:], True, B, 4 * D, D, gates, lda=D, ldb=E + D, ldc=4 * D,
                             residual=pre0[t * B:(t + 1) * B], ldr=4 * D)
                else:
                    xin = Hd[layer - 1][t] if Hd is not None else Hs[layer - 1][t + 1]
                    ops.linear(xin, W(lstm.w("weight_ih", layer), dt), lstm.w("bias_ih", layer).detach(), out=gates)
                ops.gemm(Hs[layer][t], True, W(lstm.w("weight_hh", layer), dt), True, B, 4 * D, D, gates, lda=D,
                         ldb=D, ldc=4 * D, beta=1.0, bias=lstm.w("bias_hh", layer).detach())
                hd = Hd[layer][t] if (Hd is not None and layer < L - 1) else None
                ops.lstm_cell_fwd(gates, Cs[layer][t], Cs[layer][t + 1], Hs[layer][t + 1], acts[layer][t], h_drop=hd,
                                  drop=drops[t][layer] if hd is not None else ops.NO_DROP)
            att.step_fwd(H, t, Hs[L - 1][t + 1], Hs[L - 1][t + 1], Cs[L - 1][t + 1], CtxT[t + 1])
        # LM head on b-major rows: ctx [B, T, D] (decoders.py:222-223: output_layer(dropout(context)))
        Ctxb = torch.empty(B, T, D, dtype=dt, device=dev)
        idxT = torch.arange(T, dtype=torch.int32, device=dev)
        ops.gather_rows(CtxT, idxT, Ctxb, B, T, D, B * D, D, D, T * D, x_off=B * D)
        d_out = drop()
        ctx_in = ops.dropout_apply(Ctxb.view(B * T, D), d_out) if d_out[0] > 0 else Ctxb.view(B * T, D)
        ol = m.output_layer
        wout = ol.weight._capk_pad_bf16 if dt == torch.bfloat16 else ol.weight._capk_pad_master
        logits_pad = ops.linear(ctx_in, wout, _pad_bias(ol))
        ctx.m = m
        ctx.dims = (B, T, D, E, L, V, Vp)
        ctx.saved = (features, pooled, ids_t, emb, Hs, Cs, CtxT, H, acts, Hd, drops, d_emb, d_out, ctx_in)
        ctx.logits_pad = logits_pad
        weights = H.w.permute(1, 0, 2)  # [B, T, S] (decoders.py:226-232)
        return logits_pad[:, :V].view(B, T, V), weights

    @staticmethod
    def backward(ctx, dlogits, dweights):
        m = ctx.m
        dt = m.cdtype
        B, T, D, E, L, V, Vp = ctx.dims
        features, pooled, ids_t, emb, Hs, Cs, CtxT, H, acts, Hd, drops, d_emb, d_out, ctx_in = ctx.saved
        ctx.saved = None
        dev = pooled.device
        lstm, att = m.lstm, m.attention
        ol = m.output_layer
        wout = ol.weight._capk_pad_bf16 if dt == torch.bfloat16 else ol.weight._capk_pad_master
        if dlogits is None:
            raise RuntimeError("capk LSTMDecoder: backward needs the logits gradient")
        dl = _padded_grad(dlogits, ctx.logits_pad, B * T, V, Vp)
        ctx.logits_pad = None
        ops.linear_dw(dl, ctx_in, ol.weight._capk_pad_grad)
        ops.colsum(dl, _pad_bias_grad(ol))
        dctx_b = ops.linear_dx(dl, wout)  # [B*T, D]
        if d_out[0] > 0:
            dctx_b = ops.dropout_apply(dctx_b, d_out)
        idxT = torch.arange(T, dtype=torch.int32, device=dev)
        idxB = torch.arange(B, dtype=torch.int32, device=dev)
        dCtxT = torch.empty(T, B, D, dtype=dt, device=dev)  # t-major copy of the output gradient
        ops.gather_rows(dctx_b, idxB, dCtxT, T, B, D, T * D, D, D, B * D)
        att.begin_bwd(H)
        dh = [torch.zeros(B, D, dtype=dt, device=dev) for _ in range(L)]
        dc = [torch.zeros(B, D, dtype=torch.float32, device=dev) for _ in range(L)]
        dG = [torch.empty(T, B, 4 * D, dtype=dt, device=dev) for _ in range(L)]
        dEmb = torch.empty(T, B, E, dtype=dt, device=dev)
        dctx_carry = torch.empty(B, D, dtype=dt, device=dev)
        dh_tot = torch.empty(B, D, dtype=dt, device=dev)
        w_ih0 = W(lstm.weight_ih_l0, dt)
        pair = dt == torch.bfloat16 and _PAIR and L > 1 and D % 128 == 0
        if pair:
            # layers >= 1: [dh_below | dnext] = dG [W_ih | W_hh] (N seam at D) as fp32 slabs P[l];
            # the layer below's cell sums the first half (under its dropout mask), this layer's
            # cell at t-1 the second (the top layer's: instead of the attention's dq residual)
            sb, nb = ops.pair_slabs_plan(B, 2 * D, 4 * D)
            P = [None] + [torch.empty(nb, dtype=torch.float32, device=dev) for _ in range(1, L)]
            # layer 0: [dEmb | dctx | dnext] = dG0 [W_ih0 | W_hh0] (N seam at E + D) into P0
            pair0 = (E + D) % 128 == 0
            if pair0:
                N0 = E + 2 * D
                s0, n0 = ops.pair_slabs_plan(B, N0, 4 * D)
                P0 = torch.empty(n0, dtype=torch.float32, device=dev)
        for t in range(T - 1, -1, -1):
            dctx_t = dCtxT[t] if t == T - 1 else dctx_carry
            # attention: d(query) + recurrent grad of the top layer
            att.step_bwd(H, t, dctx_t, dh_tot, dq_residual=None if pair else dh[L - 1], dc_mem_out=dc[L - 1])
            for layer in range(L - 1, -1, -1) if pair else ():
                rec = (P[layer], sb, 2 * D, D) if (layer > 0 and t < T - 1) else None
                if layer == L - 1:
                    ops.lstm_cell_bwd_slabs(acts[layer][t], Cs[layer][t], dc[layer], dG[layer][t], dh=dh_tot, rec=rec)
                else:
                    if layer == 0 and pair0:
                        rec = (P0, s0, N0, E + D) if t < T - 1 else None
                    ops.lstm_cell_bwd_slabs(acts[layer][t], Cs[layer][t], dc[layer], dG[layer][t],
                                            dh=dh[0] if (layer == 0 and not pair0) else None,
                                            up=(P[layer + 1], sb, 2 * D),
                                            drop=drops[t][layer] if Hd is not None else ops.NO_DROP, rec=rec)
                if layer > 0:
                    ops.gemm_pair_slabs(B, 2 * D, 4 * D, dG[layer][t], 4 * D, W(lstm.w("weight_ih", layer), dt), D,
                                        False, P[layer], B2=W(lstm.w("weight_hh", layer), dt), ldb2=D, n1=D)
                    continue
                if pair0:
                    ops.gemm_pair_slabs(B, N0, 4 * D, dG[0][t], 4 * D, w_ih0, E + D, False, P0,
                                        B2=W(lstm.weight_hh_l0, dt), ldb2=D, n1=E + D)
                    ops.slab_sum(P0, s0, B, N0, 0, dEmb[t])
                    if t > 0:
                        ops.slab_sum(P0, s0, B, N0, E, dctx_carry, res=dCtxT[t - 1])
                    continue
                dnext = torch.empty(B, D, dtype=dt, device=dev)
                ops.linear_dx(dG[0][t], W(lstm.weight_hh_l0, dt), out=dnext)
                ops.gemm(dG[0][t], True, w_ih0[:, :E], False, B, E, 4 * D, dEmb[t], lda=4 * D, ldb=E + D, ldc=E)
                if t > 0:
                    ops.gemm(dG[0][t], True, w_ih0[:, E:], False, B, D, 4 * D, dctx_carry, lda=4 * D, ldb=E + D,
                             ldc=D, residual=dCtxT[t - 1], ldr=D)
                dh[0] = dnext
            for layer in range(L - 1, -1, -1) if not pair else ():
                src = dh_tot if layer == L - 1 else dh_below
                ops.lstm_cell_bwd(acts[layer][t], Cs[layer][t], src, dc[layer], dG[layer][t])
                # recurrent state gradient for step t-1
                dnext = torch.empty(B, D, dtype=dt, device=dev)
                ops.linear_dx(dG[layer][t], W(lstm.w("weight_hh", layer), dt), out=dnext)
                if layer > 0:
                    # input gradient -> layer below's output at step t (dropout mask of the forward copy)
                    dh_below = torch.empty(B, D, dtype=dt, device=dev)
                    ops.gemm(dG[layer][t], True, W(lstm.w("weight_ih", layer), dt), False, B, D, 4 * D, dh_below,
                             lda=4 * D, ldb=D, ldc=D, residual=dh[layer - 1], ldr=D,
                             drop=drops[t][layer - 1] if Hd is not None else ops.NO_DROP)
                else:
                    ops.gemm(dG[0][t], True, w_ih0[:, :E], False, B, E, 4 * D, dEmb[t], lda=4 * D, ldb=E + D, ldc=E)
                    if t > 0:
                        ops.gemm(dG[0][t], True, w_ih0[:, E:], False, B, D, 4 * D, dctx_carry, lda=4 * D,
                                 ldb=E + D, ldc=D, residual=dCtxT[t - 1], ldr=D)
                dh[layer] = dnext
        if pair:  # the recurrent gradients w.r.t. the initial states
            for layer in range(1, L):
                dh[layer] = ops.slab_sum(P[layer], sb, B, 2 * D, D, torch.empty(B, D, dtype=dt, device=dev))
            if pair0:
                dh[0] = ops.slab_sum(P0, s0, B, N0, E + D, torch.empty(B, D, dtype=dt, device=dev))
        # batched weight gradients over all steps
        for layer in range(L):
            g = dG[layer].view(T * B, 4 * D)
            ops.linear_dw(g, Hs[layer][:T].reshape(T * B, D), G(lstm.w("weight_hh", layer)))
            ops.colsum(g, G(lstm.w("bias_hh", layer)))
            ops.colsum(g, G(lstm.w("bias_ih", layer)))
            if layer == 0:
                gw = G(lstm.weight_ih_l0)
                ops.gemm(g, False, emb, False, 4 * D, E, T * B, gw, lda=4 * D, ldb=E, ldc=E + D)
                ops.gemm(g, False, CtxT[:T].reshape(T * B, D), False, 4 * D, D, T * B, gw[:, E:], lda=4 * D, ldb=D,
                         ldc=E + D)
            else:
                xin = Hd[layer - 1] if Hd is not None else Hs[layer - 1][1:]
                ops.linear_dw(g, xin.reshape(T * B, D), G(lstm.w("weight_ih", layer)))
        dfeat, _ = att.finish_bwd(H, Hs[L - 1][1:].reshape(T * B, D))
        # embeddings (padding_idx row excluded, decoders.py:92-94)
        ops.zero_(G(m.embedding.weight))
        ops.embedding_bwd(ids_t, dEmb.view(T * B, E), m.pad_token_id, G(m.embedding.weight), None, 0, drop=d_emb)
        # initial states -> init_h / init_c -> pooled
        dh0 = torch.empty(B, L * D, dtype=dt, device=dev)
        dc0 = torch.empty(B, L * D, dtype=dt, device=dev)
        for layer in range(L):
            ops.copy_rows(dh[layer], dh0[:, layer * D:(layer + 1) * D])
            if dt == torch.float32:
                ops.copy_rows(dc[layer], dc0[:, layer * D:(layer + 1) * D])
            else:
                tmp = torch.empty(B, D, dtype=dt, device=dev)
                ops.cast(dc[layer], tmp)
                ops.copy_rows(tmp, dc0[:, layer * D:(layer + 1) * D])
        ops.linear_dw(dh0, pooled, G(m.init_h.weight))
        ops.colsum(dh0, G(m.init_h.bias))
        ops.linear_dw(dc0, pooled, G(m.init_c.weight))
        ops.colsum(dc0, G(m.init_c.bias))
        dpooled = ops.linear_dx(dh0, W(m.init_h.weight, dt))
        ops.linear_dx(dc0, W(m.init_c.weight, dt), out=dpooled, beta=1.0)
        return dfeat, dpooled, None, None, None


@torch.no_grad()
def lstm_greedy(m, features, pooled, max_length, start_token_id):
    """LSTMDecoder.generate (decoders.py:236-314): ids[:, t] = current token (starting
    at start_token_id), next = argmax(output_layer(ctx)); no EOS stop, no dropout."""
    dt = m.cdtype
    dev = pooled.device
    B = pooled.shape[0]
    D, E, L, V = m.hidden_dim, m.embedding_dim, m.num_layers, m.vocab_size
    lstm, att = m.lstm, m.attention
    pooled = pooled.contiguous()
    h0 = ops.linear(pooled, W(m.init_h.weight, dt), m.init_h.bias.detach())
    c0 = ops.linear(pooled, W(m.init_c.weight, dt), m.init_c.bias.detach(), out_dtype=torch.float32)
    hs = [[torch.empty(B, D, dtype=dt, device=dev) for _ in range(2)] for _ in range(L)]
    cs = [[torch.empty(B, D, dtype=torch.float32, device=dev) for _ in range(2)] for _ in range(L)]
    for layer in range(L):
        ops.copy_rows(h0[:, layer * D:(layer + 1) * D], hs[layer][0])
        ops.copy_rows(c0[:, layer * D:(layer + 1) * D], cs[layer][0])
    H = att.hoist(features, features, None, max_length)
    ids = torch.zeros(B, max_length, dtype=torch.long, device=dev)
    cur = torch.full((B,), start_token_id, dtype=torch.long, device=dev)
    ctx = [torch.zeros(B, D, dtype=dt, device=dev), torch.empty(B, D, dtype=dt, device=dev)]
    gates = torch.empty(B, 4 * D, dtype=dt, device=dev)
    act = torch.empty(B, 4 * D, dtype=dt, device=dev)
    w_ih0 = W(lstm.weight_ih_l0, dt)
    ol = m.output_layer
    wout = ol.weight._capk_pad_bf16 if dt == torch.bfloat16 else ol.weight._capk_pad_master
    for t in range(max_length):
        ids[:, t].copy_(cur)
        a, b = t % 2, (t + 1) % 2
        emb = ops.embedding_fwd(cur.view(B, 1), m.embedding.weight.detach(), None, 0, dt)
        for layer in range(L):
            if layer == 0:
                ops.linear(emb, w_ih0[:, :E], lstm.bias_ih_l0.detach(), out=gates)
                ops.gemm(ctx[a], True, w_ih0[:, E:], True, B, 4 * D, D, gates, lda=D, ldb=E + D, ldc=4 * D,
                         beta=1.0)
            else:
                ops.linear(hs[layer - 1][b], W(lstm.w("weight_ih", layer), dt), lstm.w("bias_ih", layer).detach(),
                           out=gates)
            ops.gemm(hs[layer][a], True, W(lstm.w("weight_hh", layer), dt), True, B, 4 * D, D, gates, lda=D, ldb=D,
                     ldc=4 * D, beta=1.0, bias=lstm.w("bias_hh", layer).detach())
            ops.lstm_cell_fwd(gates, cs[layer][a], cs[layer][b], hs[layer][b], act)
        att.step_fwd(H, t, hs[L - 1][b], hs[L - 1][b], cs[L - 1][b], ctx[b])
        logits = ops.linear(ctx[b], wout, _pad_bias(ol))
        ops.argmax_rows(logits, V, cur)
    return ids, {"attention_weights": H.w.permute(1, 0, 2)}


class _LSTMBank:
    """One copy of the per-row decode state: h and c of every layer ([L, R, D]; c fp32) and
    the previous attention context [R, D]."""

    def __init__(self, L, R, D, dt, dev):
        self.h = torch.empty(L, R, D, dtype=dt, device=dev)
        self.c = torch.empty(L, R, D, dtype=torch.float32, device=dev)
        self.ctx = torch.empty(R, D, dtype=dt, device=dev)
        self.device = dev


class LSTMStepRunner:
    """Incremental decode of the LSTM decoder for beam search and SCST sampling: the
    generate() loop body of decoders.py:266-303 (embed the current token, concat the
    previous context, one nn.LSTM step over all layers, attention with memory = h[-1] /
    c[-1], logits = output_layer(context)) over R = B * num_beams rows.  The image
    features, h0/c0 and the hoisted key/value projections are replicated per beam once;
    a beam reorder gathers the (h, c, context) rows of every layer into the spare bank
    (three launches) — the LSTM counterpart of the KV-cache reorder of the Transformer /
    GPT-2 runners (HF Cache.reorder_cache).  ``step(cur_len, ids, reorder)`` follows the
    capk.beam step protocol and returns [R, Vp] logits (V valid columns)."""

    def __init__(self, m, features, pooled, num_beams, max_length):
        dt = m.cdtype
        if features.dtype != dt or pooled.dtype != dt:
            raise TypeError(f"capk LSTMDecoder: feature dtype {features.dtype}/{pooled.dtype} != compute dtype {dt}")
        dev = pooled.device
        B, S, D = features.shape
        L = m.num_layers
        self.m, self.dt, self.k, self.B, self.D, self.L = m, dt, num_beams, B, D, L
        R = self.R = B * num_beams
        self.max_length = max_length
        self.rep_idx = torch.arange(R, dtype=torch.int32, device=dev) // num_beams
        pooled = pooled.contiguous()
        h0 = ops.linear(pooled, W(m.init_h.weight, dt), m.init_h.bias.detach())  # [B, L*D]
        c0 = ops.linear(pooled, W(m.init_c.weight, dt), m.init_c.bias.detach(), out_dtype=torch.float32)
        self._banks = (_LSTMBank(L, R, D, dt, dev), _LSTMBank(L, R, D, dt, dev))
        self.reset()
        b0 = self.cache
        # layer l of h0/c0 = columns [l*D, (l+1)*D) (decoders.py:122-135), replicated per beam
        ops.gather_rows(h0, self.rep_idx, b0.h, L, R, D, L * D, D, D, R * D)
        ops.gather_rows(c0, self.rep_idx, b0.c, L, R, D, L * D, D, D, R * D)
        ops.zero_(b0.ctx)  # prev_context = zeros (decoders.py:263-264)
        if num_beams > 1:
            fr = torch.empty(R, S, D, dtype=dt, device=dev)
            ops.gather_rows(features, self.rep_idx, fr, 1, R, S * D, features.stride(0), 0, S * D, 0)
        else:
            fr = features
        self.H = m.attention.hoist(fr, fr, None, max_length)
        self.gates = torch.empty(R, 4 * D, dtype=dt, device=dev)
        self.act = torch.empty(R, 4 * D, dtype=dt, device=dev)
        self.logits = torch.empty(R, m.vocab_pad, dtype=dt, device=dev)
        ol = m.output_layer
        self.wout = ol.weight._capk_pad_bf16 if dt == torch.bfloat16 else ol.weight._capk_pad_master
        self.bout = _pad_bias(ol)

    def reset(self):
        self.cache, self.spare = self._banks

    def _reorder(self, idx):
        s, d = self.cache, self.spare
        L, R, D = self.L, self.R, self.D
        ops.gather_rows(s.h, idx, d.h, L, R, D, D, R * D, D, R * D)
        ops.gather_rows(s.c, idx, d.c, L, R, D, D, R * D, D, R * D)
        ops.gather_rows(s.ctx, idx, d.ctx, 1, R, D, D, 0, D, 0)
        self.cache, self.spare = d, s

    def step(self, cur_len, ids, reorder_idx):
        m, dt, R, D, L = self.m, self.dt, self.R, self.D, self.L
        E = m.embedding_dim
        lstm = m.lstm
        if reorder_idx is not None:
            self._reorder(reorder_idx)
        src, dst = self.cache, self.spare
        t = cur_len - 1
        emb = ops.embedding_fwd(ids.view(R, 1), m.embedding.weight.detach(), None, 0, dt)
        w_ih0 = W(lstm.weight_ih_l0, dt)
        gates = self.gates
        for layer in range(L):
            if layer == 0:
                ops.linear(emb, w_ih0[:, :E], lstm.bias_ih_l0.detach(), out=gates)
                ops.gemm(src.ctx, True, w_ih0[:, E:], True, R, 4 * D, D, gates, lda=D, ldb=E + D, ldc=4 * D,
                         beta=1.0)
            else:
                ops.linear(dst.h[layer - 1], W(lstm.w("weight_ih", layer), dt), lstm.w("bias_ih", layer).detach(),
                           out=gates)
            ops.gemm(src.h[layer], True, W(lstm.w("weight_hh", layer), dt), True, R, 4 * D, D, gates, lda=D, ldb=D,
                     ldc=4 * D, beta=1.0, bias=lstm.w("bias_hh", layer).detach())
            ops.lstm_cell_fwd(gates, src.c[layer], dst.c[layer], dst.h[layer], self.act)
        m.attention.step_fwd(self.H, t, dst.h[L - 1], dst.h[L - 1], dst.c[L - 1], dst.ctx)
        ops.linear(dst.ctx, self.wout, self.bout, out=self.logits)
        self.cache, self.spare = dst, src
        return self.logits
