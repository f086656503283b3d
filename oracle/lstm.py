"""Oracle restatement of the LSTM decoder and the attention modules (SURVEY §8a rows
A6-A10).  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Parameter dicts are LSTMDecoder state dicts (``embedding.weight``,
``lstm.weight_ih_l{k}``..., ``attention.*``, ``output_layer.*``, ``init_h/init_c.*``).
"""
import torch
import torch.nn.functional as F


def _q3(q):
    """[B, D] -> ([B, 1, D], squeeze) as every module does first (attention.py:66-70)."""
    return (q[:, None], True) if q.dim() == 2 else (q, False)


def soft_attention(p, pre, q, k, v, temperature, key_pad=None):
    """SoftAttention.forward (src/models/attention.py:57-118), q [B, D] or [B, Q, D]."""
    q, sq = _q3(q)
    qp = F.linear(q, p[pre + "query_proj.weight"], p[pre + "query_proj.bias"])[:, :, None, :]
    kp = F.linear(k, p[pre + "key_proj.weight"], p[pre + "key_proj.bias"])[:, None, :, :]
    e = F.linear(torch.tanh(qp + kp), p[pre + "energy.weight"], p[pre + "energy.bias"]).squeeze(-1) / temperature
    if key_pad is not None:
        e = e.masked_fill(key_pad[:, None, :], -1e9)
    w = torch.softmax(e, -1)
    ctx = torch.matmul(w.unsqueeze(-2), v.unsqueeze(1)).squeeze(-2)
    return (ctx.squeeze(1), w.squeeze(1)) if sq else (ctx, w)


def mha_attention(p, pre, q, k, v, num_heads, temperature, key_pad=None):
    """MultiHeadAttention.forward (attention.py:142-218): scale 1/(T*sqrt(hd)),
    masked_fill(-1e9), output_proj, returned weights = mean over heads."""
    q, sq = _q3(q)
    B, Q, D = q.shape
    hd = D // num_heads

    def proj(x, name):
        return F.linear(x, p[pre + name + ".weight"], p[pre + name + ".bias"]).view(B, -1, num_heads, hd).transpose(1, 2)

    qh, kh, vh = proj(q, "query_proj"), proj(k, "key_proj"), proj(v, "value_proj")
    s = torch.matmul(qh, kh.transpose(-1, -2)) / (temperature * hd ** 0.5)
    if key_pad is not None:
        s = s.masked_fill(key_pad[:, None, None, :], -1e9)
    a = torch.softmax(s, -1)
    o = torch.matmul(a, vh).transpose(1, 2).reshape(B, Q, D)
    ctx = F.linear(o, p[pre + "output_proj.weight"], p[pre + "output_proj.bias"])
    w = a.mean(1)
    return (ctx.squeeze(1), w.squeeze(1)) if sq else (ctx, w)


def base_attention(p, pre, q, k, v, num_heads, temperature, key_pad=None):
    """AdaptiveAttention / AoA base: MHA if num_heads > 1 else SoftAttention (attention.py:236-237,308-309)."""
    if num_heads > 1:
        return mha_attention(p, pre, q, k, v, num_heads, temperature, key_pad)
    return soft_attention(p, pre, q, k, v, temperature, key_pad)


def aoa_attention(p, pre, q, k, v, num_heads, temperature, key_pad=None):
    """AttentionOnAttention.forward (attention.py:322-360)."""
    ctx, w = base_attention(p, pre + "base_attention.", q, k, v, num_heads, temperature, key_pad)
    qt = F.linear(q, p[pre + "query_proj.weight"], p[pre + "query_proj.bias"])
    cat = torch.cat([ctx, qt], -1)
    info = torch.tanh(F.linear(cat, p[pre + "info_vector_proj.0.weight"], p[pre + "info_vector_proj.0.bias"]))
    gate = torch.sigmoid(F.linear(cat, p[pre + "info_gate_proj.0.weight"], p[pre + "info_gate_proj.0.bias"]))
    return info * gate, w


def adaptive_attention(p, pre, q, k, v, num_heads, temperature, h, c, key_pad=None):
    """AdaptiveAttention.forward (attention.py:242-294): visual sentinel from the LSTM
    memory/cell state [B, D] (expanded over the Q queries), gate beta = sigmoid(W_a [ctx; s])."""
    if q.dim() == 3:
        h = h[:, None].expand(-1, q.shape[1], -1)
        c = c[:, None].expand(-1, q.shape[1], -1)
    sg = torch.sigmoid(F.linear(torch.cat([q, h], -1), p[pre + "sentinel_gate.weight"], p[pre + "sentinel_gate.bias"]))
    sent = F.linear(sg * torch.tanh(c), p[pre + "sentinel_proj.weight"], p[pre + "sentinel_proj.bias"])
    ctx, w = base_attention(p, pre + "base_attention.", q, k, v, num_heads, temperature, key_pad)
    beta = torch.sigmoid(F.linear(torch.cat([ctx, sent], -1), p[pre + "adaptive_weight.weight"],
                                  p[pre + "adaptive_weight.bias"]))
    return beta * ctx + (1 - beta) * sent, w


def standalone(kind, p, q, k, v, num_heads, temperature, key_pad=None, h=None, c=None, pre=""):
    """build_attention(cfg)(q, k, v, key_padding_mask[, memory_state, cell_state]) (attention.py:363-376)."""
    if kind == "soft":
        return soft_attention(p, pre, q, k, v, temperature, key_pad)
    if kind == "multi_head":
        return mha_attention(p, pre, q, k, v, num_heads, temperature, key_pad)
    if kind == "aoa":
        return aoa_attention(p, pre, q, k, v, num_heads, temperature, key_pad)
    if kind == "adaptive":
        return adaptive_attention(p, pre, q, k, v, num_heads, temperature, h, c, key_pad)
    raise ValueError(kind)


def attend(kind, p, q, feats, num_heads, temperature, h_top, c_top):
    pre = "attention."
    if kind == "soft":
        return soft_attention(p, pre, q, feats, feats, temperature)
    if kind == "multi_head":
        return mha_attention(p, pre, q, feats, feats, num_heads, temperature)
    if kind == "aoa":
        return aoa_attention(p, pre, q, feats, feats, num_heads, temperature)
    if kind == "adaptive":
        return adaptive_attention(p, pre, q, feats, feats, num_heads, temperature, h_top, c_top)
    raise ValueError(kind)


def lstm_step(p, x, h, c, num_layers):
    """nn.LSTM single time step, gate order i, f, g, o (torch/nn/modules/rnn.py);
    inter-layer dropout is off in eval mode."""
    hs, cs = [], []
    inp = x
    for layer in range(num_layers):
        g = (F.linear(inp, p[f"lstm.weight_ih_l{layer}"], p[f"lstm.bias_ih_l{layer}"])
             + F.linear(h[layer], p[f"lstm.weight_hh_l{layer}"], p[f"lstm.bias_hh_l{layer}"]))
        i, f, gg, o = g.chunk(4, -1)
        cn = torch.sigmoid(f) * c[layer] + torch.sigmoid(i) * torch.tanh(gg)
        hn = torch.sigmoid(o) * torch.tanh(cn)
        hs.append(hn)
        cs.append(cn)
        inp = hn
    return hs, cs


def lstm_decoder(p, feats, pooled, captions, num_layers, kind, num_heads=1, temperature=1.0):
    """LSTMDecoder.forward (src/models/decoders.py:137-234), caption_lengths=None:
    h0/c0 = init_h/init_c(pooled) (122-135); per step LSTM(cat[emb_t, ctx_{t-1}]),
    attention with query = top h, memory/cell = h[-1]/c[-1], logits = output_layer(ctx)."""
    B, T = captions.shape
    D = pooled.shape[1]
    h = list(F.linear(pooled, p["init_h.weight"], p["init_h.bias"]).view(B, num_layers, D).transpose(0, 1))
    c = list(F.linear(pooled, p["init_c.weight"], p["init_c.bias"]).view(B, num_layers, D).transpose(0, 1))
    emb = p["embedding.weight"][captions]
    ctx = torch.zeros(B, D)
    logits, weights = [], []
    for t in range(T):
        h, c = lstm_step(p, torch.cat([emb[:, t], ctx], 1), h, c, num_layers)
        ctx, w = attend(kind, p, h[-1], feats, num_heads, temperature, h[-1], c[-1])
        logits.append(F.linear(ctx, p["output_layer.weight"], p["output_layer.bias"]))
        weights.append(w)
    return torch.stack(logits, 1), torch.stack(weights, 1)


def lstm_greedy(p, feats, pooled, max_length, num_layers, kind, start_token_id, num_heads=1, temperature=1.0):
    """LSTMDecoder.generate (decoders.py:236-314): ids[:, t] = current input; next =
    argmax(output_layer(ctx)); no EOS stop."""
    B = pooled.shape[0]
    D = pooled.shape[1]
    h = list(F.linear(pooled, p["init_h.weight"], p["init_h.bias"]).view(B, num_layers, D).transpose(0, 1))
    c = list(F.linear(pooled, p["init_c.weight"], p["init_c.bias"]).view(B, num_layers, D).transpose(0, 1))
    cur = torch.full((B,), start_token_id, dtype=torch.long)
    ids = torch.zeros(B, max_length, dtype=torch.long)
    ctx = torch.zeros(B, D)
    for t in range(max_length):
        ids[:, t] = cur
        h, c = lstm_step(p, torch.cat([p["embedding.weight"][cur], ctx], 1), h, c, num_layers)
        ctx, _ = attend(kind, p, h[-1], feats, num_heads, temperature, h[-1], c[-1])
        cur = F.linear(ctx, p["output_layer.weight"], p["output_layer.bias"]).argmax(1)
    return ids
