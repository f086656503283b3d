"""Model-level parity on the GPU (north-star parity claims).

* fp32 path vs the reference-generated golden vectors (tiny ViT+Transformer,
  ragged captions with pad): logits, loss, every parameter gradient, two AdamW
  steps — all through libcapk kernels.
* fp32 path at the FULL config-3 architecture (ViT-B/16 + 6-layer Transformer,
  V = 50257) vs the CPU oracle: logits <= 1e-3 relative (BASELINE north_star).
* bf16 path (the benchmarked one) at the full architecture vs the oracle: loose
  tolerance stated in the test, plus a finite/decreasing-loss train check.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")


def _sub(p, prefix):
    return {k[len(prefix):]: v for k, v in p.items() if k.startswith(prefix)}


def _tiny_model(z, precision):
    import capk
    from capk import config as C
    from capk.models import captioning_model as cm
    from capk.models import encoders as E
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in z["meta/dims"]]
    cfg = C.Config()
    cfg.model.encoder = C.EncoderConfig(encoder_type="vit", feature_dim=D)
    cfg.model.decoder = C.DecoderConfig(decoder_type="transformer", hidden_dim=D, num_layers=Ld, num_heads=Hd)
    cfg.model.vocab_size, cfg.model.pad_token_id = V, pad
    cfg.model.bos_token_id = cfg.model.eos_token_id = pad
    arch = dict(hidden_size=D, num_hidden_layers=Le, num_attention_heads=He, intermediate_size=2 * D,
                image_size=img, patch_size=patch, num_channels=3, layer_norm_eps=1e-12)
    orig = E.VIT_ARCHS.get("google/vit-base-patch16-224")
    E.VIT_ARCHS["google/vit-base-patch16-224"] = arch
    try:
        model = cm.ImageCaptioningModel(cfg)
    finally:
        E.VIT_ARCHS["google/vit-base-patch16-224"] = orig
    sd = {k[3:]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("p0/")}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    store = capk.prepare(model, "cuda", precision)
    model.eval()  # the reference fixtures were produced with dropout off
    return model, store, cfg


@cuda
def test_golden_step_fp32(golden_dir):
    from capk.train import CapkAdamW, CombinedLoss
    z = np.load(os.path.join(golden_dir, "vit_transformer_step.npz"), allow_pickle=False)
    model, store, cfg = _tiny_model(z, "fp32")
    pad = cfg.model.pad_token_id
    images = torch.from_numpy(z["in/images"]).cuda()
    caps = torch.from_numpy(z["in/captions"]).cuda()
    out = model(images=images, captions=caps)
    np.testing.assert_allclose(out["logits"].detach().float().cpu().numpy(), z["out/logits"], rtol=1e-4, atol=2e-5)
    loss = CombinedLoss(pad)(out["logits"], caps)["total_loss"]
    np.testing.assert_allclose(float(loss), float(z["out/loss"][0]), rtol=1e-5)
    loss.backward()
    torch.cuda.synchronize()
    named = dict(model.named_parameters())
    for k in z.files:
        if k.startswith("grad/"):
            n = k[5:]
            got = named[n]._capk_grad.cpu().numpy()
            np.testing.assert_allclose(got, z[k], rtol=2e-4, atol=2e-6, err_msg=n)
    # AdamW through the flat store, two steps (same grads), lr from the schedule
    opt = CapkAdamW(store, lr=5e-3, weight_decay=0.01)
    lrs = z["out/lrs"]
    for step, tag in ((0, "p1/"), (1, "p2/")):
        opt.step(lr=float(lrs[step]))
        torch.cuda.synchronize()
        for k in z.files:
            if k.startswith(tag):
                n = k[3:]
                got, want = named[n].detach().cpu().numpy(), z[k]
                g = z["grad/" + n] if "grad/" + n in z.files else None
                if g is not None:
                    # Elements whose reference gradient is pure rounding noise (the key-projection
                    # bias of softmax attention has an analytically ZERO gradient): Adam turns noise
                    # into +-lr updates whose sign is not reproducible on any other device, so only
                    # the |update| <= lr bound per step is a meaningful check there.
                    noise = np.abs(g) < 1e-7
                    if noise.any():
                        lim = sum(float(x) for x in lrs[:step + 1]) * 1.01
                        p0 = z["p0/" + n]
                        assert np.all(np.abs(got[noise] - p0[noise]) <= lim + 1e-6), f"{tag}{n}"
                        got, want = got[~noise], want[~noise]
                # Adam divides by sqrt(v): the update of tiny-gradient elements magnifies fp32 summation-order
                # differences, so parameters are compared to 0.1 % of the summed step sizes.
                atol = 1e-3 * sum(float(x) for x in lrs[:step + 1])
                np.testing.assert_allclose(got, want, rtol=1e-5, atol=atol, err_msg=f"{tag}{n}")


@cuda
def test_golden_grads_dw_side_stream(golden_dir, monkeypatch):
    """Opt-in weight-gradient side stream (CAPK_DW_STREAM=1): the same golden gradients, read
    straight after backward() with no explicit synchronisation (the end-of-backward join must
    order them on the compute stream)."""
    from capk.models import common
    from capk.train import CombinedLoss
    monkeypatch.setattr(common, "DW_STREAM", True)
    z = np.load(os.path.join(golden_dir, "vit_transformer_step.npz"), allow_pickle=False)
    model, store, cfg = _tiny_model(z, "fp32")
    caps = torch.from_numpy(z["in/captions"]).cuda()
    out = model(images=torch.from_numpy(z["in/images"]).cuda(), captions=caps)
    CombinedLoss(cfg.model.pad_token_id)(out["logits"], caps)["total_loss"].backward()
    assert not common._DW_PENDING
    named = dict(model.named_parameters())
    for k in z.files:
        if k.startswith("grad/"):
            np.testing.assert_allclose(named[k[5:]]._capk_grad.cpu().numpy(), z[k], rtol=2e-4, atol=2e-6,
                                       err_msg=k[5:])


@cuda
def test_golden_greedy_generate_fp32(golden_dir):
    z = np.load(os.path.join(golden_dir, "vit_transformer_step.npz"), allow_pickle=False)
    model, store, cfg = _tiny_model(z, "fp32")
    images = torch.from_numpy(z["in/images"]).cuda()
    with torch.no_grad():
        ids, _ = model.generate(images=images, max_length=6)
    np.testing.assert_array_equal(ids.cpu().numpy(), z["out/greedy_ids"])


def _full_model(precision, seed=42):
    import capk
    from capk import config as C
    from capk.models import captioning_model as cm
    torch.manual_seed(seed)
    cfg = C.Config()
    cfg.model.encoder = C.EncoderConfig(encoder_type="vit")
    cfg.model.decoder = C.DecoderConfig(decoder_type="transformer")
    cfg.model.vocab_size, cfg.model.pad_token_id = 50257, 50256
    cfg.model.bos_token_id = cfg.model.eos_token_id = 50256
    model = cm.ImageCaptioningModel(cfg)
    cpu_sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    store = capk.prepare(model, "cuda", precision)
    model.eval()
    return model, store, cfg, cpu_sd


def _oracle_logits(sd, images, caps):
    from oracle import decoders as odec
    from oracle import encoders as oenc
    with torch.no_grad():
        enc = oenc.vit_encoder(_sub(sd, "encoder.model."), images, 12, 12, 16)
        return odec.transformer_decoder(_sub(sd, "decoder."), enc["features"], caps, 6, 8, 50256)


@cuda
def test_full_config3_fp32_logits_parity():
    """North-star parity: fp32 logits <= 1e-3 relative to the CPU reference path."""
    model, store, cfg, sd = _full_model("fp32")
    g = torch.Generator().manual_seed(0)
    images = torch.randn(2, 3, 224, 224, generator=g)
    caps = torch.randint(0, 50256, (2, 20), generator=torch.Generator().manual_seed(1))
    caps[1, 15:] = 50256
    with torch.no_grad():
        got = model(images=images.cuda(), captions=caps.cuda())["logits"].float().cpu()
    ref = _oracle_logits(sd, images, caps)
    rel = float((got - ref).norm() / ref.norm())
    maxrel = float((got - ref).abs().max() / ref.abs().max())
    assert rel < 1e-3 and maxrel < 1e-3, (rel, maxrel)


@cuda
def test_full_config3_bf16_logits_close():
    """bf16 storage / fp32 accumulation through 12+6 layers: stated tolerance 3e-2 relative
    (Frobenius) and argmax agreement >= 95 % against the fp32 CPU reference."""
    model, store, cfg, sd = _full_model("bf16")
    g = torch.Generator().manual_seed(0)
    images = torch.randn(2, 3, 224, 224, generator=g)
    caps = torch.randint(0, 50256, (2, 20), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        enc = model.encoder(images.cuda().bfloat16().float())
        got = model.decoder(enc, caps.cuda())["logits"].float().cpu()
    ref = _oracle_logits(sd, images, caps)
    rel = float((got - ref).norm() / ref.norm())
    agree = float((got.argmax(-1) == ref.argmax(-1)).float().mean())
    assert rel < 3e-2 and agree >= 0.95, (rel, agree)


@cuda
def test_bf16_train_steps_reduce_loss():
    from capk.train import CapkAdamW, CombinedLoss
    model, store, cfg, _ = _full_model("bf16")
    B = 8
    g = torch.Generator(device="cuda").manual_seed(0)
    images = torch.randn(B, 3, 224, 224, device="cuda", generator=g)
    caps = torch.randint(0, 50256, (B, 20), device="cuda", generator=g)
    model.train()  # decoder dropout p=0.1 active, as in the reference trainer
    opt = CapkAdamW(store, lr=1e-4)
    loss_fn = CombinedLoss(50256)
    losses = []
    for _ in range(5):
        out = model(images=images, captions=caps)
        loss = loss_fn(out["logits"], caps)["total_loss"]
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses


@cuda
@pytest.mark.parametrize("side", [False, True])
def test_deferred_finishes_bit_identical(monkeypatch, side):
    """ops.deferred_finishes -- a layer's LayerNorm weight / bias and bias column-sum finishes
    queued and launched as one kernel per stream (capk_finish_defer / capk_finish_flush_all) --
    vs every finish launched at once: a config-3 bf16 train-mode step (decoder dropout on, the
    same dropout seeds; with and without the weight-gradient side stream, whose column sums
    queue on their own stream) gives bit-identical gradients for every parameter."""
    from capk import ops
    from capk.models import common
    from capk.train import CombinedLoss
    monkeypatch.setattr(common, "DW_STREAM", side)
    model, store, cfg, _ = _full_model("bf16")
    B = 4
    g = torch.Generator(device="cuda").manual_seed(0)
    images = torch.randn(B, 3, 224, 224, device="cuda", generator=g)
    caps = torch.randint(0, 50256, (B, 20), device="cuda", generator=g)
    caps[1, 12:] = 50256
    model.train()
    loss_fn = CombinedLoss(50256)
    seed0 = common._SEED[0]
    grads = {}
    for on in (False, True):
        monkeypatch.setattr(ops, "_FIN_ON", on)
        common._SEED[0] = seed0  # the same dropout masks
        out = model(images=images, captions=caps)
        loss_fn(out["logits"], caps)["total_loss"].backward()
        torch.cuda.synchronize()
        grads[on] = {n: p._capk_grad.clone() for n, p in model.named_parameters() if getattr(p, "_capk_grad", None) is not None}
    assert grads[True].keys() == grads[False].keys() and len(grads[True]) > 200
    # (the token / position embedding gradients are scatter-added with fp32 atomics: their
    # summation order, hence their last bits, differ between any two runs)
    atomic = {"decoder.embedding.weight", "decoder.position_encoding.weight"}
    bad = [n for n in grads[True] if n not in atomic and not torch.equal(grads[True][n], grads[False][n])]
    assert not bad, bad[:10]
    for n in atomic & grads[True].keys():
        torch.testing.assert_close(grads[True][n], grads[False][n], rtol=1e-5, atol=1e-7)


@cuda
def test_weight_copies_dx_step(monkeypatch):
    """ops.WeightT on a config-3 bf16 train-mode step: every dX product on the K-major weight
    copies (MIN_ROWS lowered so the decoder's short products take them too) vs the N-major
    weights -- same gradients (per parameter within 1e-2 relative; the two operand layouts may
    pick different tile / split-K routes), and a copy-path step after an optimizer update
    matches the N-major path on the updated weights (the copies were refreshed)."""
    from capk import ops
    from capk.models import common
    from capk.train import CombinedLoss
    from capk.train.optim import CapkAdamW
    model, store, cfg, _ = _full_model("bf16")
    B = 12
    g = torch.Generator(device="cuda").manual_seed(0)
    images = torch.randn(B, 3, 224, 224, device="cuda", generator=g)
    caps = torch.randint(0, 50256, (B, 20), device="cuda", generator=g)
    model.train()
    loss_fn = CombinedLoss(50256)
    monkeypatch.setattr(ops.WeightT, "MIN_ROWS", 1)
    opt = CapkAdamW(store, lr=1e-3)

    def grads_for(on):
        monkeypatch.setattr(ops.WT, "enabled", on)
        common._SEED[0] = seed0
        out = model(images=images, captions=caps)
        loss_fn(out["logits"], caps)["total_loss"].backward()
        torch.cuda.synchronize()
        return {n: p._capk_grad.clone() for n, p in model.named_parameters() if getattr(p, "_capk_grad", None) is not None}

    def compare(a, b):
        bad = []
        for n in a:
            d = float((a[n] - b[n]).norm() / (b[n].norm() + 1e-20))
            if d > 1e-2:
                bad.append((n, d))
        assert not bad, bad[:10]

    seed0 = common._SEED[0]
    compare(grads_for(True), grads_for(False))
    assert len(ops.WT.cache) > 0
    opt.step()
    compare(grads_for(True), grads_for(False))


@cuda
def test_decoder_train_mode_dropout_matches_masked_reference(golden_dir):
    """Train-mode decoder (p=0.1 at 7 sites) vs a PyTorch reference applying the SAME masks
    (materialised with capk_dropout_mask from the intercepted per-site seeds): logits and
    every decoder gradient.  Mask index conventions: include/capk.h."""
    import math

    import torch.nn.functional as F

    from capk import ops
    from capk.models import transformer as tr
    from capk.train import CombinedLoss
    z = np.load(os.path.join(golden_dir, "vit_transformer_step.npz"), allow_pickle=False)
    model, store, cfg = _tiny_model(z, "fp32")
    dec = model.decoder
    dec.dropout_p = 0.1
    dec.train()
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in z["meta/dims"]]
    seeds = []
    orig = tr.next_seed
    tr.next_seed = lambda: (seeds.append(1000 + 7919 * len(seeds)) or seeds[-1])
    try:
        images = torch.from_numpy(z["in/images"]).cuda()
        caps = torch.from_numpy(z["in/captions"]).cuda()
        with torch.no_grad():
            feats = model.encoder(images)["features"].contiguous().clone()
        feats.requires_grad_(True)
        out = dec({"features": feats, "pooled_features": None, "attention_mask": None}, caps)
        loss = CombinedLoss(pad)(out["logits"], caps)["total_loss"]
        loss.backward()
        torch.cuda.synchronize()
    finally:
        tr.next_seed = orig
    p = 0.1
    B, T = caps.shape
    S = feats.shape[1]
    H, hd = Hd, D // Hd

    def mask(n, seed, shape):
        return ops.dropout_mask(n, p, seed).view(shape).float() / (1 - p)

    P = {n: t.detach().clone().requires_grad_(True) for n, t in dec.named_parameters()}
    fr = feats.detach().clone().requires_grad_(True)
    mem = F.linear(fr, P["visual_projection.weight"], P["visual_projection.bias"])
    si = iter(seeds)
    x = P["embedding.weight"][caps] + P["position_encoding.weight"][:T][None]
    x = x * mask(B * T * D, next(si), (B, T, D))
    tgt_pad = caps == pad

    def mha(xq, xkv, w, b, wo, bo, causal, kpad, seed, Nk):
        q = F.linear(xq, w[:D], b[:D]).view(B, T, H, hd).transpose(1, 2)
        k = F.linear(xkv, w[D:2 * D], b[D:2 * D]).view(B, Nk, H, hd).transpose(1, 2)
        v = F.linear(xkv, w[2 * D:], b[2 * D:]).view(B, Nk, H, hd).transpose(1, 2)
        s = q @ k.transpose(-1, -2) / math.sqrt(hd)
        if causal:
            s = s.masked_fill(torch.ones(T, Nk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
        if kpad is not None:
            s = s.masked_fill(kpad[:, None, None, :], float("-inf"))
        a = torch.softmax(s, -1) * mask(B * H * T * Nk, seed, (B, H, T, Nk))
        return F.linear((a @ v).transpose(1, 2).reshape(B, T, D), wo, bo)

    for i in range(Ld):
        pre = f"transformer_decoder.layers.{i}."
        s_sa, s_d1, s_ca, s_d2, s_ffn, s_d3 = [next(si) for _ in range(6)]
        y = mha(x, x, P[pre + "self_attn.in_proj_weight"], P[pre + "self_attn.in_proj_bias"],
                P[pre + "self_attn.out_proj.weight"], P[pre + "self_attn.out_proj.bias"], True, tgt_pad, s_sa, T)
        x = F.layer_norm(x + y * mask(B * T * D, s_d1, (B, T, D)), (D,), P[pre + "norm1.weight"],
                         P[pre + "norm1.bias"], 1e-5)
        y = mha(x, mem, P[pre + "multihead_attn.in_proj_weight"], P[pre + "multihead_attn.in_proj_bias"],
                P[pre + "multihead_attn.out_proj.weight"], P[pre + "multihead_attn.out_proj.bias"], False, None,
                s_ca, S)
        x = F.layer_norm(x + y * mask(B * T * D, s_d2, (B, T, D)), (D,), P[pre + "norm2.weight"],
                         P[pre + "norm2.bias"], 1e-5)
        I = P[pre + "linear1.weight"].shape[0]
        f = F.gelu(F.linear(x, P[pre + "linear1.weight"], P[pre + "linear1.bias"])) * mask(B * T * I, s_ffn,
                                                                                            (B, T, I))
        y = F.linear(f, P[pre + "linear2.weight"], P[pre + "linear2.bias"])
        x = F.layer_norm(x + y * mask(B * T * D, s_d3, (B, T, D)), (D,), P[pre + "norm3.weight"],
                         P[pre + "norm3.bias"], 1e-5)
    ref = F.linear(x, P["output_layer.weight"], P["output_layer.bias"])
    torch.testing.assert_close(out["logits"].detach(), ref.detach(), rtol=1e-4, atol=1e-5)
    F.cross_entropy(ref[:, :-1].reshape(-1, V), caps[:, 1:].reshape(-1), ignore_index=pad).backward()
    torch.testing.assert_close(feats.grad, fr.grad, rtol=1e-3, atol=1e-6)
    for n, t in dec.named_parameters():
        g = P[n].grad if P[n].grad is not None else torch.zeros_like(P[n])
        torch.testing.assert_close(t._capk_grad, g, rtol=1e-3, atol=1e-6, msg=n)


@cuda
def test_vit_pooler_vs_golden_fp32(golden_dir):
    """A1c: final LayerNorm (eps 1e-12) + tanh pooler on the CLS row (modeling_vit.py:289-301)
    vs the reference's own ViTModel pooler output (vit_transformer_step.npz out/pooled), and
    the features that feed the decoder (last_hidden_state[:, 1:], encoders.py:122)."""
    z = np.load(os.path.join(golden_dir, "vit_transformer_step.npz"), allow_pickle=False)
    model, store, cfg = _tiny_model(z, "fp32")
    images = torch.from_numpy(z["in/images"]).cuda()
    with torch.no_grad():
        enc = model.encoder(images)
    np.testing.assert_allclose(enc["pooled_features"].float().cpu().numpy(), z["out/pooled"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(enc["features"].float().cpu().numpy(), z["out/features"], rtol=1e-4, atol=1e-5)


@cuda
def test_vit_pooler_full_bf16_vs_oracle():
    """A1c in the benchmarked precision at the full ViT-B/16 shape (the tiny golden model's
    width is below the bf16 GEMM's K granularity): pooled output within 3e-2 relative of the
    fp32 oracle (oracle/encoders.py vit_model + pooler)."""
    from oracle import encoders as oenc
    model, store, cfg, sd = _full_model("bf16")
    g = torch.Generator().manual_seed(5)
    images = torch.randn(2, 3, 224, 224, generator=g)
    with torch.no_grad():
        got = model.encoder(images.cuda())["pooled_features"].float().cpu()
        ref = oenc.vit_encoder(_sub(sd, "encoder.model."), images, 12, 12, 16)["pooled_features"]
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 3e-2, rel
