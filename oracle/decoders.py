"""Oracle restatement of the caption decoders.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Parameter dicts use the reference ``TransformerDecoder`` state-dict names with
the ``decoder.`` prefix stripped (src/models/decoders.py:317-369):
``embedding.weight``, ``position_encoding.weight``,
``transformer_decoder.layers.{i}.{self_attn,multihead_attn}.{in_proj_weight,in_proj_bias,out_proj.weight,out_proj.bias}``,
``...linear1/linear2/norm1/norm2/norm3``, ``output_layer.*``, ``visual_projection.*``.
"""
import math

import torch
import torch.nn.functional as F


def mha_packed(xq, xkv, in_w, in_b, out_w, out_b, num_heads, causal=False, key_pad=None):
    """nn.MultiheadAttention forward with packed in_proj (torch/nn/functional.py
    multi_head_attention_forward): q = xq Wq^T, k/v = xkv Wk/v^T, softmax(qk^T/sqrt(hd)),
    causal float -inf mask (nn.Transformer.generate_square_subsequent_mask), bool key
    padding mask (True = pad) merged into -inf."""
    B, Tq, D = xq.shape
    Tk = xkv.shape[1]
    hd = D // num_heads
    q = F.linear(xq, in_w[:D], in_b[:D]).view(B, Tq, num_heads, hd).transpose(1, 2)
    k = F.linear(xkv, in_w[D:2 * D], in_b[D:2 * D]).view(B, Tk, num_heads, hd).transpose(1, 2)
    v = F.linear(xkv, in_w[2 * D:], in_b[2 * D:]).view(B, Tk, num_heads, hd).transpose(1, 2)
    s = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(hd)
    if causal:
        s = s.masked_fill(torch.ones(Tq, Tk, dtype=torch.bool).triu(1), float("-inf"))
    if key_pad is not None:
        s = s.masked_fill(key_pad[:, None, None, :], float("-inf"))
    a = torch.softmax(s, dim=-1)
    o = torch.matmul(a, v).transpose(1, 2).reshape(B, Tq, D)
    return F.linear(o, out_w, out_b)


def decoder_layer(p, i, x, mem, num_heads, tgt_pad=None, eps=1e-5):
    """nn.TransformerDecoderLayer.forward, post-LN branch
    (torch/nn/modules/transformer.py:1144-1153): x = norm1(x + SA(x)),
    x = norm2(x + MHA(x, mem)), x = norm3(x + linear2(gelu(linear1(x)))).
    Dropout is identity (eval / p=0 parity mode)."""
    pre = f"transformer_decoder.layers.{i}."
    D = x.shape[-1]
    sa = pre + "self_attn."
    y = mha_packed(x, x, p[sa + "in_proj_weight"], p[sa + "in_proj_bias"], p[sa + "out_proj.weight"],
                   p[sa + "out_proj.bias"], num_heads, causal=True, key_pad=tgt_pad)
    x = F.layer_norm(x + y, (D,), p[pre + "norm1.weight"], p[pre + "norm1.bias"], eps)
    ca = pre + "multihead_attn."
    y = mha_packed(x, mem, p[ca + "in_proj_weight"], p[ca + "in_proj_bias"], p[ca + "out_proj.weight"],
                   p[ca + "out_proj.bias"], num_heads)
    x = F.layer_norm(x + y, (D,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], eps)
    y = F.linear(F.gelu(F.linear(x, p[pre + "linear1.weight"], p[pre + "linear1.bias"])),
                 p[pre + "linear2.weight"], p[pre + "linear2.bias"])
    return F.layer_norm(x + y, (D,), p[pre + "norm3.weight"], p[pre + "norm3.bias"], eps)


def transformer_decoder(p, features, captions, num_layers, num_heads, pad_token_id):
    """TransformerDecoder.forward (src/models/decoders.py:371-437):
    mem = visual_projection(features) (390); memory mask dropped (D4/D5: the
    encoder mask is all ones); tgt_padding_mask = captions == pad (405);
    x = embedding(captions) + position_encoding(0..T-1) (409-414); dropout (417)
    is identity in parity mode; 6x post-LN layers (421-428); logits (431)."""
    T = captions.shape[1]
    mem = F.linear(features, p["visual_projection.weight"], p["visual_projection.bias"])
    tgt_pad = captions == pad_token_id
    x = p["embedding.weight"][captions] + p["position_encoding.weight"][:T][None]
    for i in range(num_layers):
        x = decoder_layer(p, i, x, mem, num_heads, tgt_pad)
    return F.linear(x, p["output_layer.weight"], p["output_layer.bias"])


def transformer_greedy(p, features, max_length, num_layers, num_heads, bos, eos):
    """TransformerDecoder.generate (decoders.py:439-493): greedy, starts from
    bos, re-runs the full decoder on the prefix each step (no pad mask), takes
    argmax of the last position, stops when every row emitted eos."""
    B = features.shape[0]
    mem = F.linear(features, p["visual_projection.weight"], p["visual_projection.bias"])
    ids = torch.full((B, 1), bos, dtype=torch.long)
    for _ in range(max_length - 1):
        T = ids.shape[1]
        x = p["embedding.weight"][ids] + p["position_encoding.weight"][:T][None]
        for i in range(num_layers):
            x = decoder_layer(p, i, x, mem, num_heads, None)
        logits = F.linear(x[:, -1], p["output_layer.weight"], p["output_layer.bias"])
        nxt = logits.argmax(dim=-1, keepdim=True)
        ids = torch.cat([ids, nxt], dim=1)
        if (nxt == eos).all():
            break
    return ids


def transformer_last_logits(p, mem, ids, num_layers, num_heads):
    """Last-position logits of the decoder re-run on the prefix ``ids`` [R, T] against
    projected memory ``mem`` [R, S, D] (generate's per-step computation,
    decoders.py:463-483, no pad mask) — the beam-search logits callback."""
    T = ids.shape[1]
    x = p["embedding.weight"][ids] + p["position_encoding.weight"][:T][None]
    for i in range(num_layers):
        x = decoder_layer(p, i, x, mem, num_heads, None)
    return F.linear(x[:, -1], p["output_layer.weight"], p["output_layer.bias"])


def _gelu_new(x):
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


def gpt2_decoder(p, pooled, captions, num_layers, num_heads, pad_token_id, prefix_len=10, eps=1e-5,
                 use_pad_mask=True):
    """GPT2Decoder.forward (src/models/decoders.py:554-595) with the SURVEY D7
    restatement: prefix P = image_to_prefix(pooled).view(B,10,D); every layer's past
    K = V = P split into heads (decoders.py:597-617 intent); attention mask =
    cat(ones(B,10), captions != pad); caption positions 10..10+T-1
    (modeling_gpt2.py:569-574).  GPT2Block (246-300): x += c_proj(attn(ln_1 x));
    x += mlp(ln_2 x) with Conv1D (y = x W + b, W [in, out]) and gelu_new; ln_f;
    LM head tied to wte (698).  Parameter names: the GPT2Decoder state dict minus
    ``decoder.``."""
    B, T = captions.shape
    D = p["model.transformer.wte.weight"].shape[1]
    H, hd = num_heads, D // num_heads
    P = F.linear(pooled, p["image_to_prefix.weight"], p["image_to_prefix.bias"]).view(B, prefix_len, D)
    pk = P.view(B, prefix_len, H, hd).transpose(1, 2)
    x = p["model.transformer.wte.weight"][captions] + p["model.transformer.wpe.weight"][prefix_len:prefix_len + T][None]
    keep = torch.cat([torch.ones(B, prefix_len, dtype=torch.bool), captions != pad_token_id], 1)
    if not use_pad_mask:  # generate(): HF's mask is all ones for the prompt and every generated token
        keep = torch.ones_like(keep)
    causal = torch.ones(T, prefix_len + T, dtype=torch.bool).tril(prefix_len)
    allowed = keep[:, None, None, :] & causal[None, None]
    for i in range(num_layers):
        pre = f"model.transformer.h.{i}."
        h = F.layer_norm(x, (D,), p[pre + "ln_1.weight"], p[pre + "ln_1.bias"], eps)
        qkv = h @ p[pre + "attn.c_attn.weight"] + p[pre + "attn.c_attn.bias"]
        q, k, v = (t.view(B, T, H, hd).transpose(1, 2) for t in qkv.split(D, dim=2))
        k = torch.cat([pk, k], 2)
        v = torch.cat([pk, v], 2)
        s = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(hd)
        s = s.masked_fill(~allowed, float("-inf"))
        o = torch.matmul(torch.softmax(s, -1), v).transpose(1, 2).reshape(B, T, D)
        x = x + o @ p[pre + "attn.c_proj.weight"] + p[pre + "attn.c_proj.bias"]
        h = F.layer_norm(x, (D,), p[pre + "ln_2.weight"], p[pre + "ln_2.bias"], eps)
        h = _gelu_new(h @ p[pre + "mlp.c_fc.weight"] + p[pre + "mlp.c_fc.bias"])
        x = x + h @ p[pre + "mlp.c_proj.weight"] + p[pre + "mlp.c_proj.bias"]
    x = F.layer_norm(x, (D,), p["model.transformer.ln_f.weight"], p["model.transformer.ln_f.bias"], eps)
    return x @ p["model.transformer.wte.weight"].t()
