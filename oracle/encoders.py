"""Oracle restatement of the vision encoders.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Parameters are plain dicts keyed by the reference state-dict names with the
wrapper prefix stripped (``embeddings.cls_token``, ``layers.3.mlp.fc1.weight``,
...), i.e. exactly ``ViTModel.state_dict()`` of transformers 5.15.0, which the
reference's ``ViTEncoder`` wraps as ``self.model`` (src/models/encoders.py:103-104).
"""
import math

import torch
import torch.nn.functional as F


def vit_embeddings(p, images, patch_size):
    """ViTPatchEmbeddings + ViTEmbeddings.forward
    (transformers/models/vit/modeling_vit.py:60-69, 129-161):
    Conv2d(k=s=patch) -> flatten(2).transpose(1,2) -> cat(CLS) -> + pos-emb.
    Dropout is p=0 (ViTConfig.hidden_dropout_prob)."""
    x = F.conv2d(images, p["embeddings.patch_embeddings.projection.weight"],
                 p["embeddings.patch_embeddings.projection.bias"], stride=patch_size)
    x = x.flatten(2).transpose(1, 2)
    cls = p["embeddings.cls_token"].expand(x.shape[0], -1, -1)
    x = torch.cat([cls, x], dim=1)
    return x + p["embeddings.position_embeddings"]


def mha_self(x, wq, bq, wk, bk, wv, bv, wo, bo, num_heads, causal=False, key_pad=None):
    """Scaled-dot-product self attention with separate q/k/v projections
    (ViTAttention, modeling_vit.py:207-238 + eager/sdpa 164-189): scale 1/sqrt(hd),
    non-causal, no mask for ViT."""
    B, N, D = x.shape
    hd = D // num_heads
    q = F.linear(x, wq, bq).view(B, N, num_heads, hd).transpose(1, 2)
    k = F.linear(x, wk, bk).view(B, N, num_heads, hd).transpose(1, 2)
    v = F.linear(x, wv, bv).view(B, N, num_heads, hd).transpose(1, 2)
    s = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(hd)
    if causal:
        s = s.masked_fill(torch.ones(N, N, dtype=torch.bool).triu(1), float("-inf"))
    if key_pad is not None:
        s = s.masked_fill(key_pad[:, None, None, :], float("-inf"))
    a = torch.softmax(s, dim=-1)
    o = torch.matmul(a, v).transpose(1, 2).reshape(B, N, D)
    return F.linear(o, wo, bo)


def vit_layer(p, i, x, num_heads, eps):
    """ViTLayer.forward (modeling_vit.py:266-286), pre-LN:
    x += o_proj(SDPA(LN_before(x))); x += fc2(GELU_erf(fc1(LN_after(x))))."""
    pre = f"layers.{i}."
    D = x.shape[-1]
    h = F.layer_norm(x, (D,), p[pre + "layernorm_before.weight"], p[pre + "layernorm_before.bias"], eps)
    a = pre + "attention."
    x = x + mha_self(h, p[a + "q_proj.weight"], p[a + "q_proj.bias"], p[a + "k_proj.weight"],
                     p[a + "k_proj.bias"], p[a + "v_proj.weight"], p[a + "v_proj.bias"],
                     p[a + "o_proj.weight"], p[a + "o_proj.bias"], num_heads)
    h = F.layer_norm(x, (D,), p[pre + "layernorm_after.weight"], p[pre + "layernorm_after.bias"], eps)
    h = F.gelu(F.linear(h, p[pre + "mlp.fc1.weight"], p[pre + "mlp.fc1.bias"]))
    return x + F.linear(h, p[pre + "mlp.fc2.weight"], p[pre + "mlp.fc2.bias"])


def vit_model(p, images, num_layers, num_heads, patch_size, eps=1e-12):
    """ViTModel.forward (modeling_vit.py:336-381): embeddings -> layers -> final
    layernorm (348) -> ViTPooler tanh(dense(h[:,0])) (289-301)."""
    x = vit_embeddings(p, images, patch_size)
    for i in range(num_layers):
        x = vit_layer(p, i, x, num_heads, eps)
    D = x.shape[-1]
    seq = F.layer_norm(x, (D,), p["layernorm.weight"], p["layernorm.bias"], eps)
    pooled = torch.tanh(F.linear(seq[:, 0], p["pooler.dense.weight"], p["pooler.dense.bias"]))
    return seq, pooled


def _proj(x, proj):
    """encoders.py:108-112 / 199-203: nn.Linear(hidden, feature_dim) when the sizes differ
    (proj = (weight, bias)), nn.Identity otherwise (proj = None)."""
    return x if proj is None else F.linear(x, proj[0], proj[1])


def vit_encoder(p, images, num_layers, num_heads, patch_size, eps=1e-12, proj=None):
    """ViTEncoder.forward (src/models/encoders.py:118-137): features drop CLS
    (122), proj applied to features and pooled (123, 127), all-ones mask
    (130-131; restated as None = no key padding)."""
    seq, pooled = vit_model(p, images, num_layers, num_heads, patch_size, eps)
    return {"features": _proj(seq[:, 1:], proj), "pooled_features": _proj(pooled, proj), "attention_mask": None}


def clip_vision(p, images, num_layers, num_heads, patch_size, eps=1e-5):
    """CLIPVisionModel.forward (transformers 5.15 modeling_clip.py): embeddings
    (179-196: bias-free Conv2d patch, class_embedding, position_embedding) ->
    pre_layrnorm (642) -> pre-LN layers (355-395: quick_gelu MLP) -> last_hidden_state;
    pooled = post_layernorm(last_hidden_state[:, 0]) (650-651).  Parameter names are
    the (flattened) CLIPVisionModel state dict."""
    x = F.conv2d(images, p["embeddings.patch_embedding.weight"], None, stride=patch_size)
    x = x.flatten(2).transpose(1, 2)
    B, _, D = x.shape
    cls = p["embeddings.class_embedding"].expand(B, 1, -1)
    x = torch.cat([cls, x], 1) + p["embeddings.position_embedding.weight"][None]
    x = F.layer_norm(x, (D,), p["pre_layrnorm.weight"], p["pre_layrnorm.bias"], eps)
    for i in range(num_layers):
        pre = f"encoder.layers.{i}."
        h = F.layer_norm(x, (D,), p[pre + "layer_norm1.weight"], p[pre + "layer_norm1.bias"], eps)
        a = pre + "self_attn."
        x = x + mha_self(h, p[a + "q_proj.weight"], p[a + "q_proj.bias"], p[a + "k_proj.weight"],
                         p[a + "k_proj.bias"], p[a + "v_proj.weight"], p[a + "v_proj.bias"],
                         p[a + "out_proj.weight"], p[a + "out_proj.bias"], num_heads)
        h = F.layer_norm(x, (D,), p[pre + "layer_norm2.weight"], p[pre + "layer_norm2.bias"], eps)
        h = F.linear(h, p[pre + "mlp.fc1.weight"], p[pre + "mlp.fc1.bias"])
        h = h * torch.sigmoid(1.702 * h)  # quick_gelu
        x = x + F.linear(h, p[pre + "mlp.fc2.weight"], p[pre + "mlp.fc2.bias"])
    pooled = F.layer_norm(x[:, 0], (D,), p["post_layernorm.weight"], p["post_layernorm.bias"], eps)
    return x, pooled


def clip_encoder(p, images, num_layers, num_heads, patch_size, eps=1e-5, proj=None):
    """CLIPEncoder.forward (src/models/encoders.py:209-230): features =
    proj(last_hidden_state[:, 1:]) (no post-LN), pooled = proj(pooler_output)."""
    seq, pooled = clip_vision(p, images, num_layers, num_heads, patch_size, eps)
    return {"features": _proj(seq[:, 1:], proj), "pooled_features": _proj(pooled, proj), "attention_mask": None}


# ------------------------------------------------------------------ ResNet (A3) --
def _conv_bn(p, pre, x, stride, training, relu, state=None, momentum=0.1, eps=1e-5):
    """ResNetConvLayer.forward (transformers/models/resnet/modeling_resnet.py:39-71):
    Conv2d(bias=False, padding=k//2) -> BatchNorm2d -> ReLU (or identity).
    `state` (dict of running buffers, updated in place in training mode) defaults to p."""
    w = p[pre + "convolution.weight"]
    x = F.conv2d(x, w, None, stride=stride, padding=w.shape[-1] // 2)
    st = p if state is None else state
    rm, rv = st[pre + "normalization.running_mean"], st[pre + "normalization.running_var"]
    x = F.batch_norm(x, rm, rv, p[pre + "normalization.weight"], p[pre + "normalization.bias"], training,
                     momentum, eps)
    return F.relu(x) if relu else x


def resnet_model(p, images, hidden_sizes, depths, training=True, state=None, downsample_in_first_stage=False):
    """ResNetModel.forward (modeling_resnet.py:291-330), bottleneck layers (v1.5, stride on
    the 3x3: downsample_in_bottleneck=False): returns (last_hidden_state, pooler_output)."""
    x = _conv_bn(p, "embedder.embedder.", images, 2, training, True, state)  # ResNetEmbeddings 74-92
    x = F.max_pool2d(x, 3, 2, 1)
    for si, depth in enumerate(depths):
        for li in range(depth):
            pre = f"encoder.stages.{si}.layers.{li}."
            stride = (2 if (si > 0 or downsample_in_first_stage) else 1) if li == 0 else 1
            # ResNetBottleNeckLayer.forward (143-190)
            h = _conv_bn(p, pre + "layer.0.", x, 1, training, True, state)
            h = _conv_bn(p, pre + "layer.1.", h, stride, training, True, state)
            h = _conv_bn(p, pre + "layer.2.", h, 1, training, False, state)
            if pre + "shortcut.convolution.weight" in p:
                r = _conv_bn(p, pre + "shortcut.", x, stride, training, False, state)  # ResNetShortCut 95-110
            else:
                r = x
            x = F.relu(h + r)
    return x, F.adaptive_avg_pool2d(x, (1, 1))


def resnet_encoder(p, images, hidden_sizes, depths, training=True, state=None):
    """ResNetEncoder.forward (src/models/encoders.py:60-91) with the SURVEY §0.1 D6
    restatement: features = proj(map.flatten(2).transpose(1,2)), pooled = proj(pool.flatten(1));
    proj = Identity when hidden_sizes[-1] == feature_dim (no "proj.*" entries, encoders.py:50-54)."""
    last, pool = resnet_model(_strip(p, "model."), images, hidden_sizes, depths, training,
                              None if state is None else _strip(state, "model."))
    pr = (p["proj.weight"], p["proj.bias"]) if "proj.weight" in p else None
    feats = _proj(last.flatten(2).transpose(1, 2), pr)
    pooled = _proj(pool.flatten(1), pr)
    return {"features": feats, "pooled_features": pooled}


def _strip(p, prefix):
    return {k[len(prefix):]: v for k, v in p.items() if k.startswith(prefix)}


# ------------------------------------------------------------------- QFormer ----
def qformer(p, features, num_layers, num_heads, eps=1e-5):
    """QFormer.forward (src/models/captioning_model.py:202-245) in eval mode: the learnable
    queries through `num_layers` norm_first nn.TransformerEncoderLayer blocks
    (x += SA(LN1 x); x += W2 GELU(W1 LN2 x)), then `num_layers` norm_first
    nn.TransformerDecoderLayer blocks cross-attending the (vision_proj-ed) features
    (x += SA(LN1 x); x += MHA(LN2 x, mem); x += FFN(LN3 x)); torch's layer math
    (torch/nn/modules/transformer.py) with packed in_proj weights.  The encoders' all-ones
    mask becomes an additive 0 key mask (no masking)."""
    from .decoders import mha_packed
    B = features.shape[0]
    D = p["query_tokens"].shape[-1]
    x = p["query_tokens"].expand(B, -1, -1)
    mem = F.linear(features, p["vision_proj.weight"], p["vision_proj.bias"]) if "vision_proj.weight" in p \
        else features

    def ln(t, pre):
        return F.layer_norm(t, (D,), p[pre + ".weight"], p[pre + ".bias"], eps)

    def ffn(t, pre):
        return F.linear(F.gelu(F.linear(t, p[pre + "linear1.weight"], p[pre + "linear1.bias"])),
                        p[pre + "linear2.weight"], p[pre + "linear2.bias"])

    def mha(q, kv, pre):
        return mha_packed(q, kv, p[pre + "in_proj_weight"], p[pre + "in_proj_bias"], p[pre + "out_proj.weight"],
                          p[pre + "out_proj.bias"], num_heads)

    for i in range(num_layers):
        pre = f"encoder.layers.{i}."
        h = ln(x, pre + "norm1")
        x = x + mha(h, h, pre + "self_attn.")
        x = x + ffn(ln(x, pre + "norm2"), pre)
    for i in range(num_layers):
        pre = f"decoder.layers.{i}."
        h = ln(x, pre + "norm1")
        x = x + mha(h, h, pre + "self_attn.")
        x = x + mha(ln(x, pre + "norm2"), mem, pre + "multihead_attn.")
        x = x + ffn(ln(x, pre + "norm3"), pre)
    return x


# ---------------------------------------------------------------------- Swin ----
def _swin_rel_index(ws):
    """SwinRelativePositionBias._create_relative_position_index (modeling_swin.py:350-365):
    (r_i - r_j + ws - 1) * (2ws - 1) + (c_i - c_j + ws - 1) for window tokens i, j."""
    r = torch.arange(ws).repeat_interleave(ws)
    c = torch.arange(ws).repeat(ws)
    return (r[:, None] - r[None, :] + ws - 1) * (2 * ws - 1) + (c[:, None] - c[None, :] + ws - 1)


def _swin_windows(x, ws):
    """window_partition (modeling_swin.py:486-496): [B,H,W,C] -> [B*nW, ws*ws, C]."""
    B, H, W, C = x.shape
    x = x.view(B, H // ws, ws, W // ws, ws, C).permute(0, 1, 3, 2, 4, 5)
    return x.reshape(-1, ws * ws, C)


def _swin_unwindows(w, ws, B, H, W):
    C = w.shape[-1]
    x = w.view(B, H // ws, W // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5)
    return x.reshape(B, H, W, C)


def _swin_shift_mask(H, W, ws, shift):
    """SwinLayer.get_attn_mask (modeling_swin.py:584-607): -100 between tokens of different
    cyclic-shift regions of a window (regions [0, n-ws), [n-ws, n-shift), [n-shift, n) per axis)."""
    img = torch.zeros(1, H, W, 1)
    cnt = 0
    for hs in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
        for wsl in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
            img[:, hs, wsl, :] = cnt
            cnt += 1
    mw = _swin_windows(img, ws).squeeze(-1)
    m = mw[:, None, :] - mw[:, :, None]
    return m.masked_fill(m != 0, -100.0)


def swin_block(p, pre, x, H, W, num_heads, ws, shift, eps=1e-5, keep=None):
    """SwinLayer.forward (modeling_swin.py:529-574): x [B, H*W, C] natural order.
    keep [B] (optional): SwinDropPath's per-sample factor floor(U + keep_prob)/keep_prob on the
    attention branch (the MLP branch has no drop path in this transformers version)."""
    B, L, C = x.shape
    if min(H, W) <= ws:  # set_shift_and_window_size
        ws, shift = min(H, W), 0
    hd = C // num_heads
    h = F.layer_norm(x, (C,), p[pre + "layernorm_before.weight"], p[pre + "layernorm_before.bias"], eps)
    h = h.view(B, H, W, C)
    if shift:
        h = torch.roll(h, (-shift, -shift), dims=(1, 2))
    win = _swin_windows(h, ws)
    nWB, N, _ = win.shape
    a = pre + "attention."
    q = F.linear(win, p[a + "q_proj.weight"], p[a + "q_proj.bias"]).view(nWB, N, num_heads, hd).transpose(1, 2)
    k = F.linear(win, p[a + "k_proj.weight"], p[a + "k_proj.bias"]).view(nWB, N, num_heads, hd).transpose(1, 2)
    v = F.linear(win, p[a + "v_proj.weight"], p[a + "v_proj.bias"]).view(nWB, N, num_heads, hd).transpose(1, 2)
    s = torch.matmul(q, k.transpose(-1, -2)) * hd ** -0.5
    table = p[a + "relative_position_bias.relative_position_bias_table"]
    bias = table[_swin_rel_index(ws).reshape(-1)].view(N, N, -1).permute(2, 0, 1)
    s = s + bias.unsqueeze(0)
    if shift:
        m = _swin_shift_mask(H, W, ws, shift)
        nW = m.shape[0]
        s = (s.view(B, nW, num_heads, N, N) + m[None, :, None]).view(nWB, num_heads, N, N)
    o = torch.matmul(torch.softmax(s, dim=-1), v).transpose(1, 2).reshape(nWB, N, C)
    o = F.linear(o, p[a + "o_proj.weight"], p[a + "o_proj.bias"])
    o = _swin_unwindows(o, ws, B, H, W)
    if shift:
        o = torch.roll(o, (shift, shift), dims=(1, 2))
    o = o.reshape(B, L, C)
    if keep is not None:
        o = o * keep.view(B, 1, 1)
    x = x + o
    h = F.layer_norm(x, (C,), p[pre + "layernorm_after.weight"], p[pre + "layernorm_after.bias"], eps)
    h = F.linear(F.gelu(F.linear(h, p[pre + "mlp.fc1.weight"], p[pre + "mlp.fc1.bias"])),
                 p[pre + "mlp.fc2.weight"], p[pre + "mlp.fc2.bias"])
    return x + h


def swin_merge(p, pre, x, H, W):
    """SwinPatchMerging.forward (modeling_swin.py:309-326): 2x2 neighbours concatenated in the
    order (row 0, col 0), (1, 0), (0, 1), (1, 1) -> LN(4C) -> Linear(4C -> 2C, no bias)."""
    B, L, C = x.shape
    x = x.view(B, H, W, C)
    x = torch.cat([x[:, 0::2, 0::2], x[:, 1::2, 0::2], x[:, 0::2, 1::2], x[:, 1::2, 1::2]], dim=-1)
    x = x.reshape(B, -1, 4 * C)
    x = F.layer_norm(x, (4 * C,), p[pre + "norm.weight"], p[pre + "norm.bias"], 1e-5)
    return F.linear(x, p[pre + "reduction.weight"])


def swin_model(p, images, depths, heads, patch_size=4, window_size=7, eps=1e-5, keep=None):
    """SwinModel.forward (modeling_swin.py:849-900) up to the final layernorm:
    patch conv -> embeddings.norm -> stages (blocks alternate shift 0 / ws//2, patch merge
    between stages) -> layernorm.  Returns [B, h*w, C_last].  keep: optional list of [B]
    drop-path factors, one per block in order."""
    x = F.conv2d(images, p["embeddings.patch_embeddings.projection.weight"],
                 p["embeddings.patch_embeddings.projection.bias"], stride=patch_size)
    B, C, H, W = x.shape
    x = x.flatten(2).transpose(1, 2)
    x = F.layer_norm(x, (C,), p["embeddings.norm.weight"], p["embeddings.norm.bias"], 1e-5)
    bi = 0
    for s, d in enumerate(depths):
        for i in range(d):
            pre = f"encoder.layers.{s}.blocks.{i}."
            x = swin_block(p, pre, x, H, W, heads[s], window_size, 0 if i % 2 == 0 else window_size // 2, eps,
                           None if keep is None else keep[bi])
            bi += 1
        if s < len(depths) - 1:
            x = swin_merge(p, f"encoder.layers.{s}.downsample.", x, H, W)
            H, W = H // 2, W // 2
    C = x.shape[-1]
    return F.layer_norm(x, (C,), p["layernorm.weight"], p["layernorm.bias"], eps)


def swin_encoder(p, images, depths, heads, patch_size=4, window_size=7, keep=None):
    """SwinEncoder.forward (src/models/encoders.py:165-182): features = proj(last_hidden_state)
    (proj = Linear when hidden_size != feature_dim, else identity), pooled = features.mean(1).
    p: the encoder's state dict ("model.*", "proj.*")."""
    x = swin_model(_strip(p, "model."), images, depths, heads, patch_size, window_size, keep=keep)
    if "proj.weight" in p:
        x = F.linear(x, p["proj.weight"], p["proj.bias"])
    return x, x.mean(dim=1)
