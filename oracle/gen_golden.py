"""Generate golden vectors by running the REFERENCE code itself (build container only).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  This script imports
/root/reference as the package ``src.*`` and runs its own
forward / loss / backward / optimizer code on tiny random-init models built
from HF config classes (no ``from_pretrained``: there is no network).  The
§0.1 restatements are applied as wrappers *around* reference objects, never as
edits:

* D4/D5: the encoder's float all-ones ``attention_mask`` is replaced by None
  before it reaches the decoder (semantically identical: no padded image tokens).
* Encoders are constructed with ``__new__`` and their HF ``.model`` assigned
  (the reference __init__ calls ``from_pretrained``).

Outputs: ``tests/golden/<case>.npz`` (inputs, parameters, outputs, grads,
optimizer-updated params).  Only data is committed; the reference never travels.

Usage:  python oracle/gen_golden.py            (writes every case)
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def _import_reference():
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import src.config as rconfig  # noqa: F401
    import src.models.encoders as renc
    import src.models.decoders as rdec
    import src.models.attention as ratt
    import src.models.captioning_model as rcap
    import src.train.losses as rloss
    import src.train.trainer as rtrain
    return types.SimpleNamespace(config=rconfig, enc=renc, dec=rdec, att=ratt, cap=rcap,
                                 loss=rloss, train=rtrain)


def _np(t):
    return t.detach().cpu().numpy().astype(np.float32) if t.is_floating_point() else t.detach().cpu().numpy()


def case_vit_transformer(R):
    """Config 3 path (ViT + TransformerDecoder + MHA): full CE train step with
    the reference's ImageCaptioningModel.forward, CombinedLoss, backward,
    CaptioningTrainer._create_optimizer (AdamW groups) and _create_scheduler."""
    from transformers import ViTConfig, ViTModel
    torch.manual_seed(1234)
    D, L_enc, H_enc, L_dec, H_dec, V = 32, 2, 2, 2, 4, 61
    pad = V - 1  # GPT-2 convention pad == eos == bos (src/main.py:160-168)
    vcfg = ViTConfig(hidden_size=D, num_hidden_layers=L_enc, num_attention_heads=H_enc,
                     intermediate_size=2 * D, image_size=32, patch_size=8, num_channels=3)
    enc = R.enc.ViTEncoder.__new__(R.enc.ViTEncoder)
    nn.Module.__init__(enc)
    enc.model = ViTModel(vcfg)
    enc.feature_dim = D
    enc.proj = nn.Identity()
    dcfg = R.config.DecoderConfig(decoder_type=R.config.DecoderType.TRANSFORMER, hidden_dim=D,
                                  num_layers=L_dec, num_heads=H_dec, dropout=0.1, max_length=50)
    dec = R.dec.TransformerDecoder(dcfg, vocab_size=V, pad_token_id=pad, bos_token_id=pad,
                                   eos_token_id=pad)
    cfg = R.config.Config.__new__(R.config.Config)
    model = R.cap.ImageCaptioningModel.__new__(R.cap.ImageCaptioningModel)
    nn.Module.__init__(model)
    model.config = cfg
    model.encoder = enc
    model.decoder = dec
    # D4/D5 restatement: all-ones float mask -> None, applied around the reference forward.
    orig_fwd = enc.forward
    enc.forward = lambda images: {**orig_fwd(images), "attention_mask": None}
    model.eval()  # dropout off: parity mode (SURVEY §7 "Dropout/sampling RNG")

    B, T = 3, 7
    images = torch.randn(B, 3, 32, 32)
    captions = torch.randint(0, V - 1, (B, T))
    captions[1, 5:] = pad  # ragged caption: padded tail (ignored by CE, masked keys)
    captions[2, 6] = pad
    params0 = {n: p.detach().clone() for n, p in model.named_parameters()}

    out = model(images=images, captions=captions, caption_lengths=None)
    logits = out["logits"]
    loss_fn = R.loss.CombinedLoss(pad_token_id=pad)
    loss = loss_fn(logits=logits, targets=captions)["total_loss"]
    loss.backward()
    grads = {n: (p.grad.detach().clone() if p.grad is not None else None)
             for n, p in model.named_parameters()}

    # Optimizer + scheduler through the reference trainer's own factory methods.
    tcfg = R.config.TrainingConfig(learning_rate=5e-3, warmup_steps=2, num_epochs=1)
    fake = types.SimpleNamespace(model=model, config=types.SimpleNamespace(training=tcfg),
                                 train_loader=list(range(10)))
    opt = R.train.CaptioningTrainer._create_optimizer(fake)
    fake.optimizer = opt
    sched = R.train.CaptioningTrainer._create_scheduler(fake)
    lrs = [sched.get_last_lr()[0]]
    opt.step()
    sched.step()
    lrs.append(sched.get_last_lr()[0])
    params1 = {n: p.detach().clone() for n, p in model.named_parameters()}
    # second step with the same grads (grads unchanged: no zero_grad, no new backward)
    opt.step()
    sched.step()
    lrs.append(sched.get_last_lr()[0])
    params2 = {n: p.detach().clone() for n, p in model.named_parameters()}
    for _ in range(5):
        sched.step()
        lrs.append(sched.get_last_lr()[0])

    # greedy generate (TransformerDecoder.generate) from the step-0 weights
    with torch.no_grad():
        model.load_state_dict(params0, strict=False)
        gen_ids, _ = model.generate(images=images, max_length=6)

    arrs = {
        "meta/dims": np.array([D, L_enc, H_enc, L_dec, H_dec, V, pad, 8, 32], dtype=np.int64),
        "in/images": _np(images), "in/captions": _np(captions),
        "out/logits": _np(logits), "out/loss": _np(loss.reshape(1)),
        "out/features": _np(enc(images)["features"]),
        "out/pooled": _np(enc(images)["pooled_features"]),
        "out/lrs": np.array(lrs, dtype=np.float64),
        "out/greedy_ids": _np(gen_ids),
        "opt/no_decay": np.array([n for n in params0 if any(k in n for k in ("bias", "LayerNorm.weight"))]),
    }
    for n in params0:
        arrs["p0/" + n] = _np(params0[n])
        arrs["p1/" + n] = _np(params1[n])
        arrs["p2/" + n] = _np(params2[n])
        if grads[n] is not None:
            arrs["grad/" + n] = _np(grads[n])
    return arrs


def _d7_wrap(R, dec, prefix_len=10):
    """SURVEY D7 restatement applied around the reference GPT2Decoder: the prefix
    becomes a per-layer K = V = image_prefix.view(B,10,H,hd).transpose(1,2) cache
    (the "simplified placeholder" intent of decoders.py:597-617) and the attention
    mask gains the 10 always-visible prefix slots."""
    from transformers import DynamicCache
    cfg = dec.model.config
    H = cfg.n_head

    def prefix_cache(prefix_embeds):
        B, P, D = prefix_embeds.shape
        kv = prefix_embeds.view(B, P, H, D // H).transpose(1, 2)
        cache = DynamicCache()
        for layer in range(cfg.n_layer):
            cache.update(kv, kv, layer)
        return cache

    dec._create_prefix_past_key_values = prefix_cache
    inner = dec.model.forward

    def fwd(*a, **kw):
        ids, am = kw.get("input_ids"), kw.get("attention_mask")
        if am is not None and ids is not None and am.shape[1] == ids.shape[1]:
            kw["attention_mask"] = torch.cat([torch.ones(am.shape[0], prefix_len, dtype=am.dtype), am], 1)
        return inner(*a, **kw)

    dec.model.forward = fwd


def case_clip_gpt2(R):
    """Config 4 path (CLIP-ViT + GPT2Decoder; AoA inert, D15): CE train step through
    the reference's ImageCaptioningModel.forward (CLIPEncoder, GPT2Decoder with the D7
    prefix restatement), CombinedLoss and backward; eval mode (dropout off)."""
    from transformers import CLIPVisionConfig, CLIPVisionModel
    torch.manual_seed(4321)
    D, Le, He, Ld, Hd, V = 64, 2, 2, 2, 2, 61
    pad = V - 1
    ccfg = CLIPVisionConfig(hidden_size=D, num_hidden_layers=Le, num_attention_heads=He, intermediate_size=2 * D,
                            image_size=64, patch_size=32, num_channels=3)
    enc = R.enc.CLIPEncoder.__new__(R.enc.CLIPEncoder)
    nn.Module.__init__(enc)
    enc.model = CLIPVisionModel(ccfg)
    enc.feature_dim = D
    enc.proj = nn.Identity()
    dcfg = R.config.DecoderConfig(decoder_type=R.config.DecoderType.GPT2, pretrained_model_name=None, hidden_dim=D,
                                  num_layers=Ld, num_heads=Hd, dropout=0.1, max_length=40)
    dec = R.dec.GPT2Decoder(dcfg, vocab_size=V, pad_token_id=pad, bos_token_id=pad, eos_token_id=pad)
    _d7_wrap(R, dec)
    cfg = R.config.Config.__new__(R.config.Config)
    model = R.cap.ImageCaptioningModel.__new__(R.cap.ImageCaptioningModel)
    nn.Module.__init__(model)
    model.config = cfg
    model.encoder = enc
    model.decoder = dec
    orig_fwd = enc.forward
    enc.forward = lambda images: {**orig_fwd(images), "attention_mask": None}
    model.eval()

    B, T = 3, 7
    images = torch.randn(B, 3, 64, 64)
    captions = torch.randint(0, V - 1, (B, T))
    captions[0, 0] = pad  # bos
    captions[1, 5:] = pad
    captions[2, 6] = pad
    params0 = {n: p.detach().clone() for n, p in model.named_parameters()}
    out = model(images=images, captions=captions, caption_lengths=None)
    logits = out["logits"]
    loss = R.loss.CombinedLoss(pad_token_id=pad)(logits=logits, targets=captions)["total_loss"]
    loss.backward()
    feats = enc(images)
    arrs = {
        "meta/dims": np.array([D, Le, He, Ld, Hd, V, pad, 32, 64], dtype=np.int64),
        "in/images": _np(images), "in/captions": _np(captions),
        "out/logits": _np(logits), "out/loss": _np(loss.reshape(1)),
        "out/features": _np(feats["features"]), "out/pooled": _np(feats["pooled_features"]),
    }
    for n, p in model.named_parameters():
        arrs["p0/" + n] = _np(params0[n])
        if p.grad is not None:
            arrs["grad/" + n] = _np(p.grad)
    return arrs


def case_lstm_attention(R):
    """LSTMDecoder (decoders.py:70-314) with each attention type of attention.py
    (soft with temperature 0.7, multi_head, aoa, adaptive; heads 4): teacher-forced
    forward (caption_lengths=None, D10), CombinedLoss, backward (eval mode).  Encoder
    features are plain leaf tensors so their gradients are recorded too.  D3: the
    AttentionConfig receives hidden_dim as build_decoder's restatement does."""
    torch.manual_seed(777)
    D, L, V, B, T, S = 64, 2, 53, 3, 6, 7
    pad = V - 1
    arrs = {"meta/dims": np.array([D, L, V, B, T, S, pad], dtype=np.int64)}
    feats = torch.randn(B, S, D)
    pooled = torch.randn(B, D)
    caps = torch.randint(0, V - 1, (B, T))
    caps[1, 4:] = pad
    arrs["in/features"], arrs["in/pooled"], arrs["in/captions"] = _np(feats), _np(pooled), _np(caps)
    variants = [("soft", R.config.AttentionType.SOFT, 1, 0.7), ("multi_head", R.config.AttentionType.MULTI_HEAD, 4, 1.0),
                ("aoa", R.config.AttentionType.AOA, 4, 1.0), ("adaptive", R.config.AttentionType.ADAPTIVE, 4, 1.0),
                ("adaptive_soft", R.config.AttentionType.ADAPTIVE, 1, 1.0)]
    for name, at, heads, temp in variants:
        torch.manual_seed(1000 + len(name))
        dcfg = R.config.DecoderConfig(decoder_type=R.config.DecoderType.LSTM, hidden_dim=D, num_layers=L,
                                      num_heads=heads, dropout=0.1, max_length=50)
        acfg = R.config.AttentionConfig(attention_type=at, num_heads=heads, temperature=temp)
        acfg.hidden_dim = D  # D3
        dec = R.dec.LSTMDecoder(dcfg, acfg, vocab_size=V, pad_token_id=pad)
        dec.eval()
        f = feats.clone().requires_grad_(True)
        pl = pooled.clone().requires_grad_(True)
        out = dec({"features": f, "pooled_features": pl, "attention_mask": None}, caps, None)
        loss = R.loss.CombinedLoss(pad_token_id=pad)(logits=out["logits"], targets=caps)["total_loss"]
        loss.backward()
        pre = name + "/"
        arrs[pre + "logits"] = _np(out["logits"])
        arrs[pre + "attention_weights"] = _np(out["attention_weights"])
        arrs[pre + "loss"] = _np(loss.reshape(1))
        arrs[pre + "dfeatures"] = _np(f.grad)
        arrs[pre + "dpooled"] = _np(pl.grad)
        with torch.no_grad():
            ids, info = dec.generate({"features": feats, "pooled_features": pooled, "attention_mask": None}, 6,
                                     start_token_id=pad)
        arrs[pre + "greedy_ids"] = _np(ids)
        for n, p in dec.named_parameters():
            arrs[pre + "p0/" + n] = _np(p)
            if p.grad is not None:
                arrs[pre + "grad/" + n] = _np(p.grad)
    return arrs


def case_attention_standalone(R):
    """The AttentionMechanism drop-in contract (attention.py:12-35) of every module that
    build_attention returns (attention.py:363-376), called standalone:
    soft (T 0.7), multi_head (4 heads), aoa and adaptive over an MHA base (4 heads) and over
    a soft base (1 head).  Three query forms per module:
      q1  query [B, D] (2-D), key is value (one tensor), no mask;
      q1m query [B, 1, D], distinct key / value, key_padding_mask;
      qT  query [B, T=20, D], distinct key / value, key_padding_mask.
    Loss = <context, gc> + <weights, gw> (the returned weights are differentiable in the
    reference, MHA's head mean included); grads of query, key, value, memory_state,
    cell_state (adaptive) and every parameter."""
    D, B, S, T = 64, 3, 7, 20
    arrs = {"meta/dims": np.array([D, B, S, T], dtype=np.int64)}
    mask = torch.zeros(B, S, dtype=torch.bool)
    mask[1, S - 2:] = True
    mask[2, S - 4:] = True
    arrs["in/mask"] = _np(mask)
    variants = [("soft", R.config.AttentionType.SOFT, 1, 0.7), ("multi_head", R.config.AttentionType.MULTI_HEAD, 4, 1.0),
                ("aoa", R.config.AttentionType.AOA, 4, 1.0), ("aoa_soft", R.config.AttentionType.AOA, 1, 1.0),
                ("adaptive", R.config.AttentionType.ADAPTIVE, 4, 1.3),
                ("adaptive_soft", R.config.AttentionType.ADAPTIVE, 1, 1.0)]
    torch.manual_seed(4242)
    inputs = {}
    for form, Q in (("q1", 0), ("q1m", 1), ("qT", T)):
        q = torch.randn(B, D) if Q == 0 else torch.randn(B, Q, D)
        k = torch.randn(B, S, D)
        v = k if form == "q1" else torch.randn(B, S, D)
        h, c = torch.randn(B, D), torch.randn(B, D)
        gc = torch.randn(B, D) if Q == 0 else torch.randn(B, Q, D)
        gw = torch.randn(B, S) if Q == 0 else torch.randn(B, Q, S)
        inputs[form] = (q, k, v, h, c, gc, gw, None if form == "q1" else mask)
        for n, t in (("query", q), ("key", k), ("value", v), ("memory_state", h), ("cell_state", c), ("gc", gc),
                     ("gw", gw)):
            arrs[f"in/{form}/{n}"] = _np(t)
    for name, at, heads, temp in variants:
        torch.manual_seed(2000 + 7 * len(name) + heads)
        acfg = R.config.AttentionConfig(attention_type=at, num_heads=heads, temperature=temp)
        acfg.hidden_dim = D  # D3
        mod = R.att.build_attention(acfg)
        for n, p in mod.named_parameters():
            arrs[f"{name}/p0/{n}"] = _np(p)
        for form, (q, k, v, h, c, gc, gw, m) in inputs.items():
            mod.zero_grad(set_to_none=True)
            ql = q.clone().requires_grad_(True)
            kl = k.clone().requires_grad_(True)
            vl = kl if form == "q1" else v.clone().requires_grad_(True)
            hl = h.clone().requires_grad_(True)
            cl = c.clone().requires_grad_(True)
            kw = {"memory_state": hl, "cell_state": cl} if name.startswith("adaptive") else {}
            ctx, w = mod(ql, kl, vl, m, **kw)
            ((ctx * gc).sum() + (w * gw).sum()).backward()
            pre = f"{name}/{form}/"
            arrs[pre + "context"], arrs[pre + "weights"] = _np(ctx), _np(w)
            arrs[pre + "dquery"], arrs[pre + "dkey"] = _np(ql.grad), _np(kl.grad)
            if form != "q1":
                arrs[pre + "dvalue"] = _np(vl.grad)
            if kw:
                arrs[pre + "dmemory_state"], arrs[pre + "dcell_state"] = _np(hl.grad), _np(cl.grad)
            for n, p in mod.named_parameters():
                arrs[pre + "grad/" + n] = _np(p.grad) if p.grad is not None else np.zeros(tuple(p.shape), np.float32)
    return arrs


def case_resnet_lstm(R):
    """Config 2 path (ResNet + LSTMDecoder + soft attention), TRAIN mode (BatchNorm on batch
    statistics, running buffers updated) with decoder dropout 0 so the step is deterministic.
    The encoder is the reference's HF ``ResNetModel`` + ``proj`` with the SURVEY §0.1 D6
    restatement applied around it (encoders.py:60-91 raises as written):
    features = proj(last_hidden_state.flatten(2).transpose(1,2)), pooled = proj(pooler.flatten(1)).
    Tiny bottleneck net: stages 16->32 (stride-1 projection shortcut, identity shortcut),
    ->64, ->64, ->128 (stride-2 projection shortcuts), 64x64 images -> 2x2 maps."""
    from transformers import ResNetConfig, ResNetModel
    torch.manual_seed(4242)
    D, L, V, B, T = 64, 2, 53, 3, 6
    pad = V - 1
    rcfg = ResNetConfig(num_channels=3, embedding_size=16, hidden_sizes=[32, 64, 64, 128], depths=[2, 1, 2, 1],
                        layer_type="bottleneck", hidden_act="relu", downsample_in_first_stage=False,
                        downsample_in_bottleneck=False)
    enc = R.enc.ResNetEncoder.__new__(R.enc.ResNetEncoder)
    nn.Module.__init__(enc)
    enc.model = ResNetModel(rcfg)
    enc.feature_dim = D
    enc.proj = nn.Linear(rcfg.hidden_sizes[-1], D)

    def d6_forward(images):
        out = enc.model(images)
        feats = enc.proj(out.last_hidden_state.flatten(2).transpose(1, 2))
        pooled = enc.proj(out.pooler_output.flatten(1))
        return {"features": feats, "pooled_features": pooled, "attention_mask": None}  # D4/D5

    enc.forward = d6_forward
    dcfg = R.config.DecoderConfig(decoder_type=R.config.DecoderType.LSTM, hidden_dim=D, num_layers=L, num_heads=1,
                                  dropout=0.0, max_length=50)
    acfg = R.config.AttentionConfig(attention_type=R.config.AttentionType.SOFT, num_heads=1, temperature=1.0)
    acfg.hidden_dim = D  # D3
    dec = R.dec.LSTMDecoder(dcfg, acfg, vocab_size=V, pad_token_id=pad)
    model = R.cap.ImageCaptioningModel.__new__(R.cap.ImageCaptioningModel)
    nn.Module.__init__(model)
    model.config = R.config.Config.__new__(R.config.Config)
    model.encoder = enc
    model.decoder = dec
    model.train()
    images = torch.randn(B, 3, 64, 64)
    captions = torch.randint(0, V - 1, (B, T))
    captions[2, 4:] = pad
    state0 = {n: t.detach().clone() for n, t in model.state_dict().items()}
    out = model(images=images, captions=captions, caption_lengths=None)
    loss = R.loss.CombinedLoss(pad_token_id=pad)(logits=out["logits"], targets=captions)["total_loss"]
    loss.backward()
    with torch.no_grad():
        feats_train = enc(images)  # second train-mode pass: updates running stats again
        enc.eval()
        feats_eval = enc(images)
    state1 = {n: t.detach().clone() for n, t in model.state_dict().items()}
    arrs = {"meta/dims": np.array([D, L, V, B, T, pad, 64], dtype=np.int64),
            "in/images": _np(images), "in/captions": _np(captions),
            "out/logits": _np(out["logits"]), "out/loss": _np(loss.reshape(1)),
            "out/features_train": _np(feats_train["features"]), "out/pooled_train": _np(feats_train["pooled_features"]),
            "out/features_eval": _np(feats_eval["features"]), "out/pooled_eval": _np(feats_eval["pooled_features"])}
    for n, t in state0.items():
        arrs["s0/" + n] = _np(t)
    for n, t in state1.items():
        if not n.endswith(("weight", "bias")) or "running" in n:
            arrs["s2/" + n] = _np(t)  # buffers after two train-mode passes
    for n, p in model.named_parameters():
        if p.grad is not None:
            arrs["grad/" + n] = _np(p.grad)
    return arrs


def _digest(arrs, key, t, full_max=65536):
    """Large tensors travel as a digest: the first 4096 flat values + sum / abs-sum / norm."""
    a = _np(t).astype(np.float64)
    if a.size <= full_max:
        arrs[key] = a.astype(np.float32)
        return
    flat = a.reshape(-1)
    arrs[key + "@head"] = flat[:4096].astype(np.float32)
    arrs[key + "@stats"] = np.array([flat.sum(), np.abs(flat).sum(), np.sqrt((flat * flat).sum())])


def case_legacy_decoder(R):
    """Config 1 decoder (models/decoder.py Decoder, use_bert=False) + the train.py step
    (train.py:84-112): packed CE + ((1 - sum_t alpha)^2).mean(), backward, grad clamp +-5,
    Adam(lr 4e-4) — run by the reference's own code (import needs a stub
    `pytorch_pretrained_bert` module: it is imported at module level but unused when
    use_bert=False).  Dropout p=0.5 is set to 0 for a deterministic step.  The decoder dims
    are hard-coded (2048/512/512), so its parameters are NOT stored: they are re-created
    from the seed by the build's Decoder (same construction/RNG order) and pinned by
    digests; large gradients / updated weights travel as digests (_digest)."""
    import importlib
    stub = types.ModuleType("pytorch_pretrained_bert")
    stub.BertTokenizer = stub.BertModel = object
    sys.modules.setdefault("pytorch_pretrained_bert", stub)
    sys.path.insert(0, os.path.join(REF, "models"))
    try:
        rdec = importlib.import_module("models.decoder")
    finally:
        sys.path.pop(0)
    from torch.nn.utils.rnn import pack_padded_sequence
    V, B, S = 40, 4, 16
    lengths = [7, 6, 6, 4]
    torch.manual_seed(2024)
    dec = rdec.Decoder(V, False, "cpu")
    dec.dropout.p = 0.0
    dec.train()
    torch.manual_seed(7)
    enc_out = torch.randn(B, 4, 4, 2048).requires_grad_(True)
    caps = torch.zeros(B, max(lengths), dtype=torch.long)
    for b, L in enumerate(lengths):
        caps[b, 0] = 1
        caps[b, 1:L - 1] = torch.randint(3, V, (L - 2,))
        caps[b, L - 1] = 2
    arrs = {"meta/dims": np.array([V, B, S], dtype=np.int64), "in/lengths": np.array(lengths, dtype=np.int64),
            "in/encoder_out": _np(enc_out), "in/captions": _np(caps)}
    for n, p in dec.named_parameters():
        _digest(arrs, "p0/" + n, p, full_max=0)
    scores, caps_sorted, decode_lengths, alphas = dec(enc_out, caps, lengths)
    arrs["out/predictions"], arrs["out/alphas"] = _np(scores), _np(alphas)
    sp = pack_padded_sequence(scores, decode_lengths, batch_first=True)[0]
    tg = pack_padded_sequence(caps_sorted[:, 1:], decode_lengths, batch_first=True)[0]
    loss = nn.CrossEntropyLoss()(sp, tg)  # D12: train.py never defines `criterion`
    loss = loss + ((1. - alphas.sum(dim=1)) ** 2).mean()
    opt = torch.optim.Adam(params=dec.parameters(), lr=4e-4)
    opt.zero_grad()
    loss.backward()
    arrs["out/loss"] = _np(loss.reshape(1))
    arrs["out/dencoder_out"] = _np(enc_out.grad)
    for n, p in dec.named_parameters():
        _digest(arrs, "grad/" + n, p.grad)
    for group in opt.param_groups:  # train.py:105-110
        for param in group["params"]:
            if param.grad is not None:
                param.grad.data.clamp_(-5., 5.)
    opt.step()
    for n, p in dec.named_parameters():
        _digest(arrs, "p1/" + n, p, full_max=0)
    return arrs


def case_qformer(R):
    """The reference's BLIP-2 style QFormer (src/models/captioning_model.py:153-245): two
    norm_first nn.TransformerEncoder layers over the learnable queries, then two
    nn.TransformerDecoder layers cross-attending the vision features; eval mode (dropout
    off), with the all-ones vision mask the encoders return (-> additive 0 key mask)."""
    torch.manual_seed(77)
    D, Q, H, S, B = 32, 4, 4, 6, 2
    qf = R.cap.QFormer(query_dim=D, vision_dim=D, num_queries=Q, num_layers=2, num_heads=H, dropout=0.1)
    qf.eval()
    feats = torch.randn(B, S, D, requires_grad=True)
    mask = torch.ones(B, S)
    out = qf(feats, mask)["queries"]
    g = torch.randn_like(out)
    (out * g).sum().backward()
    arrs = {"meta/dims": np.array([D, Q, H, S, B], dtype=np.int64), "in/features": _np(feats),
            "in/grad_out": _np(g), "out/queries": _np(out), "out/dfeatures": _np(feats.grad)}
    for n, p in qf.named_parameters():
        arrs["p0/" + n] = _np(p)
        arrs["grad/" + n] = _np(p.grad)
    return arrs


def case_swin_encoder(R):
    """The reference's SwinEncoder.forward (src/models/encoders.py:140-182) on a random-init
    transformers SwinModel: 112x112 input -> stages at 28x28 (16 windows, shifted blocks),
    14x14 (4 windows, shifted) and 7x7 (window clamped to the resolution, no shift); proj
    Linear(128 -> 48) since hidden_size != feature_dim; features.mean pooling.  Eval mode
    (SwinDropPath off).  The relative-position tables (zero at HF init) are randomised so
    the bias path is exercised.  Loss = <features, gf> + <pooled, gp> with fixed random
    gf, gp, so every parameter receives a gradient through both outputs."""
    from transformers import SwinConfig, SwinModel
    torch.manual_seed(4321)
    scfg = SwinConfig(image_size=112, patch_size=4, embed_dim=32, depths=[2, 2, 2], num_heads=[1, 2, 4],
                      window_size=7, drop_path_rate=0.1)
    enc = R.enc.SwinEncoder.__new__(R.enc.SwinEncoder)
    nn.Module.__init__(enc)
    enc.model = SwinModel(scfg)
    enc.feature_dim = 48
    enc.proj = nn.Linear(enc.model.config.hidden_size, enc.feature_dim)  # encoders.py:153-158
    with torch.no_grad():
        for n, p in enc.named_parameters():
            if n.endswith("relative_position_bias_table"):
                p.normal_(0.0, 0.5)
            elif n.endswith("norm.weight") or "layernorm" in n and n.endswith("weight"):
                p.add_(0.1 * torch.randn_like(p))
    enc.eval()
    B = 2
    images = torch.randn(B, 3, 112, 112)
    out = enc(images)
    feats, pooled = out["features"], out["pooled_features"]
    gf = torch.randn_like(feats)
    gp = torch.randn_like(pooled)
    ((feats * gf).sum() + (pooled * gp).sum()).backward()
    arrs = {"meta/dims": np.array([112, 4, 32, 7, 48, B], dtype=np.int64),
            "meta/depths": np.array([2, 2, 2], dtype=np.int64), "meta/heads": np.array([1, 2, 4], dtype=np.int64),
            "in/images": _np(images), "in/gf": _np(gf), "in/gp": _np(gp),
            "out/features": _np(feats), "out/pooled": _np(pooled), "out/mask": _np(out["attention_mask"])}
    for n, p in enc.named_parameters():
        arrs["p0/" + n] = _np(p)
        arrs["grad/" + n] = _np(p.grad)
    return arrs


CASES = {"vit_transformer_step": case_vit_transformer, "qformer_step": case_qformer, "clip_gpt2_step": case_clip_gpt2,
         "lstm_attention": case_lstm_attention, "attention_standalone": case_attention_standalone,
         "resnet_lstm_step": case_resnet_lstm,
         "legacy_decoder_step": case_legacy_decoder, "swin_encoder": case_swin_encoder}


def main(names=None):
    R = _import_reference()
    os.makedirs(OUT, exist_ok=True)
    for name, fn in CASES.items():
        if names and name not in names:
            continue
        arrs = fn(R)
        path = os.path.join(OUT, name + ".npz")
        np.savez_compressed(path, **arrs)
        print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB, {len(arrs)} arrays)")


if __name__ == "__main__":
    main(sys.argv[1:])
