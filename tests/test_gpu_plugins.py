"""Plugin options beyond the benchmarked configurations, each against the oracle (GPU):

* encoder projections (src/models/encoders.py:50-54, 108-112, 199-203): ViT / CLIP with
  hidden_size != feature_dim (features and pooled both projected, gradients of every
  parameter), ResNet with hidden_sizes[-1] == feature_dim (identity: the map rows and the
  average-pooled map);
* GPT-2 ``generate(num_beams=1)`` (decoders.py:619-654 forwards num_beams to HF generate:
  greedy search) vs oracle/beam.py greedy_search over the oracle GPT-2 (pinned to HF by
  tests/test_oracle_beam.py) — sequences bit-exact;
* LSTM decoder beam search (HF beam semantics for every decoder) vs
  oracle/beam.py over the oracle LSTM decoder for every attention variant — sequences and
  beam indices bit-exact;
* SCST with the LSTM decoder (trainer.py:338-438): sampled ids vs the oracle sampler over
  the oracle LSTM, loss and every decoder gradient vs autograd of the oracle;
* the CLI train path: ``capk.main(["--steps", "2", ...])`` through the trainer, then a
  checkpoint round trip.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _rel(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _sub(p, prefix):
    return {k[len(prefix):]: v for k, v in p.items() if k.startswith(prefix)}


# ------------------------------------------------------------ encoder projections ---
@cuda
@pytest.mark.parametrize("family", ["vit", "clip"])
def test_token_encoder_projection_fp32(family):
    import capk
    from capk import config as C
    from capk.models import encoders as E
    from oracle import encoders as oenc
    torch.manual_seed(3)
    D, F, Le, He, patch, img = 64, 40, 2, 4, 16, 48
    arch = dict(hidden_size=D, num_hidden_layers=Le, num_attention_heads=He, intermediate_size=2 * D,
                image_size=img, patch_size=patch, num_channels=3,
                layer_norm_eps=1e-12 if family == "vit" else 1e-5)
    cfg = C.EncoderConfig(encoder_type=family, feature_dim=F)
    enc = (E.ViTEncoder if family == "vit" else E.CLIPEncoder)(cfg, arch=arch)
    assert isinstance(enc.proj, torch.nn.Linear) and enc.proj.weight.shape == (F, D)
    sd = {k: v.detach().clone() for k, v in enc.state_dict().items()}
    capk.prepare(enc, "cuda", "fp32")
    g = torch.Generator().manual_seed(4)
    B = 3
    images = torch.randn(B, 3, img, img, generator=g)
    out = enc(images.cuda())
    N = (img // patch) ** 2
    assert out["features"].shape == (B, N, F) and out["pooled_features"].shape == (B, F)
    gf = torch.randn(B, N, F, generator=g)
    gp = torch.randn(B, F, generator=g)
    ((out["features"] * gf.cuda()).sum() + (out["pooled_features"] * gp.cuda()).sum()).backward()
    p = {k: v.float().requires_grad_(True) for k, v in sd.items()}
    fn = oenc.vit_encoder if family == "vit" else oenc.clip_encoder
    eps = {"eps": 1e-12} if family == "vit" else {}
    ref = fn(_sub(p, "model."), images, Le, He, patch, proj=(p["proj.weight"], p["proj.bias"]), **eps)
    ((ref["features"] * gf).sum() + (ref["pooled_features"] * gp).sum()).backward()
    assert _rel(out["features"], ref["features"]) < 1e-4
    assert _rel(out["pooled_features"], ref["pooled_features"]) < 1e-4
    checked = 0
    gmax = max(float(p[n].grad.abs().max()) for n, _ in enc.named_parameters() if p[n].grad is not None)
    for n, prm in enc.named_parameters():
        gref = p[n].grad
        if gref is None:
            continue
        # fp32 kernels vs fp32 autograd: 1e-3 relative per parameter, or within 1e-5 of the
        # largest gradient of the model (parameters whose gradient is ~0, e.g. an LN bias
        # before a mean-free path)
        err = float((prm._capk_grad.cpu() - gref).norm())
        assert err <= 1e-3 * float(gref.norm()) or float((prm._capk_grad.cpu() - gref).abs().max()) <= 1e-5 * gmax, n
        checked += 1
    assert checked >= 2 + 8 * Le


@cuda
def test_resnet_identity_projection_fp32():
    """hidden_sizes[-1] == feature_dim -> proj = nn.Identity (encoders.py:50-54): features =
    the flattened final map, pooled = its average (SURVEY D6 restatement), with gradients."""
    import capk
    from capk import config as C
    from capk.models import encoders as E
    from oracle import encoders as oenc
    torch.manual_seed(5)
    arch = dict(num_channels=3, embedding_size=16, hidden_sizes=(32, 64), depths=(1, 1),
                downsample_in_first_stage=False, downsample_in_bottleneck=False)
    enc = E.ResNetEncoder(C.EncoderConfig(encoder_type="resnet", feature_dim=64), arch=arch)
    assert isinstance(enc.proj, torch.nn.Identity)
    sd = {k: v.detach().clone() for k, v in enc.state_dict().items()}
    capk.prepare(enc, "cuda", "fp32")
    g = torch.Generator().manual_seed(6)
    images = torch.randn(2, 3, 64, 64, generator=g)
    out = enc(images.cuda())
    ref = oenc.resnet_encoder({k: v.clone() for k, v in sd.items()}, images, [32, 64], [1, 1], training=True)
    assert out["features"].shape == ref["features"].shape
    assert _rel(out["features"], ref["features"]) < 1e-4
    assert _rel(out["pooled_features"], ref["pooled_features"]) < 1e-4
    gf = torch.randn(*ref["features"].shape, generator=g)
    gp = torch.randn(*ref["pooled_features"].shape, generator=g)
    ((out["features"] * gf.cuda()).sum() + (out["pooled_features"] * gp.cuda()).sum()).backward()
    p = {k: (v.float().clone().requires_grad_(True) if "running" not in k and "num_batches" not in k else v.clone())
         for k, v in sd.items()}
    ref = oenc.resnet_encoder(p, images, [32, 64], [1, 1], training=True, state={k: v.clone() for k, v in sd.items()})
    ((ref["features"] * gf).sum() + (ref["pooled_features"] * gp).sum()).backward()
    checked = 0
    for n, prm in enc.named_parameters():  # BatchNorm affine gradients (natural layout) of every block
        if "normalization" not in n:
            continue
        torch.testing.assert_close(prm._capk_grad.cpu(), p[n].grad, rtol=1e-3,
                                   atol=1e-3 * float(p[n].grad.abs().max()) + 1e-7, msg=lambda m: f"{n}: {m}")
        checked += 1
    assert checked >= 10


# ------------------------------------------------------------------- GPT-2 greedy ---
def _clip_gpt2(precision):
    from test_gpu_config4 import _model
    return _model(precision)


@cuda
def test_gpt2_greedy_generate_vs_oracle_fp32():
    from oracle import decoders as odec
    from oracle import encoders as oenc
    from oracle.beam import greedy_search
    z, model, store, cfg = _clip_gpt2("fp32")
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in z["meta/dims"]]
    images = torch.from_numpy(z["in/images"])
    with torch.no_grad():
        ids, info = model.generate(images=images.cuda(), max_length=12, num_beams=1)
    assert info == {}
    sd = {k: v.detach().cpu().float() for k, v in model.state_dict().items()}
    enc = oenc.clip_encoder(_sub(sd, "encoder.model."), images, Le, He, patch)
    p = _sub(sd, "decoder.")
    pooled = enc["pooled_features"]

    def fn(seqs):
        with torch.no_grad():
            return odec.gpt2_decoder(p, pooled, seqs, Ld, Hd, pad, use_pad_mask=False)[:, -1]

    ref = greedy_search(fn, images.shape[0], 12, eos=pad, pad=pad, bos=pad)
    assert torch.equal(ids.cpu(), ref), (ids.cpu(), ref)


# --------------------------------------------------------------------- LSTM beam ----
LSTM_VARIANTS = {"soft": ("soft", 1, 0.7), "multi_head": ("multi_head", 4, 1.0), "aoa": ("aoa", 4, 1.0),
                 "adaptive": ("adaptive", 4, 1.0)}


def _lstm(name, precision, eos):
    import capk
    from capk import config as C
    from capk.models.decoders import build_decoder
    z = np.load(os.path.join(GOLD, "lstm_attention.npz"), allow_pickle=False)
    D, L, V, B, T, S, pad = [int(x) for x in z["meta/dims"]]
    kind, heads, temp = LSTM_VARIANTS[name]
    dec = build_decoder(C.DecoderConfig(decoder_type="lstm", hidden_dim=D, num_layers=L, num_heads=heads, dropout=0.1),
                        C.AttentionConfig(attention_type=kind, num_heads=heads, temperature=temp), V, pad, pad, eos)
    pre = name + "/p0/"
    sd = {k[len(pre):]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith(pre)}
    dec.load_state_dict(sd, strict=True)
    capk.prepare(dec, "cuda", precision)
    dec.eval()
    p = {k: v.float() for k, v in sd.items()}
    return z, dec, p, (D, L, V, B, T, S, pad, kind, heads, temp)


@cuda
@pytest.mark.parametrize("name", sorted(LSTM_VARIANTS))
def test_lstm_beam_search_vs_oracle_fp32(name):
    from oracle import lstm as olstm
    from oracle.beam import beam_search as oracle_beam
    k, Lmax = 3, 9
    z, dec, p, (D, L, V, B, T, S, pad, kind, heads, temp) = _lstm(name, "fp32", eos=5)
    feats = torch.from_numpy(z["in/features"])
    pooled = torch.from_numpy(z["in/pooled"])
    with torch.no_grad():
        ids, info = dec.generate({"features": feats.cuda(), "pooled_features": pooled.cuda()}, Lmax, num_beams=k,
                                 start_token_id=1)
    fr, pr = feats.repeat_interleave(k, 0), pooled.repeat_interleave(k, 0)

    def fn(seqs):
        with torch.no_grad():
            return olstm.lstm_decoder(p, fr, pr, seqs, L, kind, heads, temp)[0][:, -1]

    ref = oracle_beam(fn, B, k, Lmax, bos=1, eos=5, pad=pad)
    assert torch.equal(ids.cpu(), ref["sequences"]), (ids.cpu(), ref["sequences"])
    assert torch.equal(info["beam_indices"].cpu(), ref["beam_indices"])
    torch.testing.assert_close(info["sequences_scores"].cpu(), ref["sequences_scores"], rtol=1e-4, atol=1e-5)


@cuda
def test_lstm_beam_full_size_bf16_runs():
    """Config-2 decoder geometry (768 x 6, 49 keys, V = 50257), beam 5 in bf16: runs and
    returns well-formed sequences (bf16 ties make exact agreement with fp32 unspecified)."""
    import capk
    from capk import config as C
    from capk.models.decoders import build_decoder
    torch.manual_seed(21)
    V, pad = 50257, 50256
    dec = build_decoder(C.DecoderConfig(decoder_type="lstm", hidden_dim=768, num_layers=6),
                        C.AttentionConfig(attention_type="soft"), V, pad, pad, pad)
    capk.prepare(dec, "cuda", "bf16")
    dec.eval()
    g = torch.Generator(device="cuda").manual_seed(2)
    feats = torch.randn(16, 49, 768, device="cuda", generator=g).bfloat16()
    pooled = torch.randn(16, 768, device="cuda", generator=g).bfloat16()
    with torch.no_grad():
        ids, info = dec.generate({"features": feats, "pooled_features": pooled}, 20, num_beams=5)
    assert ids.shape[0] == 16 and 2 <= ids.shape[1] <= 20
    assert bool((ids[:, 0] == 1).all()) and bool(((ids >= 0) & (ids < V)).all())
    assert torch.isfinite(info["sequences_scores"]).all()


# --------------------------------------------------------------------- LSTM SCST ----
@cuda
def test_lstm_scst_sampling_and_update_vs_oracle():
    import torch.nn.functional as F
    from capk.train import CapkAdamW
    from capk.train.scst import cider_d, pg_targets, sample_captions, scst_step, strip_special
    from oracle import lstm as olstm
    from oracle import scst as oscst

    class _Enc(torch.nn.Module):  # fixed encoder features (the decoder is what is under test)
        def __init__(self, f, q):
            super().__init__()
            self.f, self.q = f, q

        def forward(self, images):
            return {"features": self.f, "pooled_features": self.q, "attention_mask": None}

    class _Model(torch.nn.Module):
        def __init__(self, enc, dec):
            super().__init__()
            self.encoder, self.decoder = enc, dec

    eos = 5
    z, dec, p, (D, L, V, B, T, S, pad, kind, heads, temp) = _lstm("soft", "fp32", eos=eos)
    feats = torch.from_numpy(z["in/features"]).cuda()
    pooled = torch.from_numpy(z["in/pooled"]).cuda()
    model = _Model(_Enc(feats, pooled), dec)
    from capk.params import store_of
    store = store_of(dec)
    seed, Lmax = 77, 8
    with torch.no_grad():
        ids, logp = sample_captions(dec, {"features": feats, "pooled_features": pooled}, Lmax, seed=seed)
    fc, qc = feats.cpu(), pooled.cpu()
    oids = torch.full((B, 1), dec.bos_token_id, dtype=torch.long)
    olp = []
    with torch.no_grad():
        for t in range(Lmax - 1):
            lg = olstm.lstm_decoder(p, fc, qc, oids, L, kind, heads, temp)[0][:, -1]
            picks = [oscst.sample_row(lg[r].numpy(), seed, t, r) for r in range(B)]
            nxt = torch.tensor([tok for tok, _, _ in picks])
            olp.append([lp for _, lp, _ in picks])
            oids = torch.cat([oids, nxt[:, None]], 1)
            if bool((nxt == eos).all()):
                break
    assert torch.equal(ids.cpu(), oids), (ids.cpu(), oids)
    np.testing.assert_allclose(logp.cpu().numpy(), np.array(olp, dtype=np.float32).T, rtol=1e-4, atol=1e-4)
    refs = [[[3, 5, 7, 9], [6, 7]], [[1, 2, 3]], [[4, 4, 8, 15, 16]], [[2, 4, 6]]]
    while len(refs) < B:
        refs.append([[2, 4, 6]])
    refs = refs[:B]
    opt = CapkAdamW(store, lr=0.0, weight_decay=0.0)
    loss, rs, rb = scst_step(model, None, refs, opt, lr=0.0, seed=seed, max_length=Lmax)
    bos = dec.bos_token_id
    samp = [strip_special(r, eos, pad, bos) for r in ids.cpu().tolist()]
    with torch.no_grad():  # the reference baseline: LSTM greedy from start token 1 (decoders.py:236-314)
        base_ids, _ = dec.generate({"features": feats, "pooled_features": pooled}, Lmax)
    base = [strip_special(r, eos, pad, bos) for r in base_ids.cpu().tolist()]
    adv = torch.tensor(cider_d(samp, refs) - cider_d(base, refs), dtype=torch.float32)
    assert float(adv.abs().sum()) > 0
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    logits = olstm.lstm_decoder(pr, fc, qc, ids.cpu(), L, kind, heads, temp)[0]
    tgt = pg_targets(ids.cpu(), eos)
    lp = F.log_softmax(logits[:, :-1], -1).gather(-1, tgt[:, 1:].clamp(min=0)[..., None])[..., 0]
    mask = (tgt[:, 1:] != -100).float()
    ref = -(lp * adv[:, None] * mask).sum() / mask.sum()
    ref.backward()
    torch.testing.assert_close(loss.cpu(), ref.detach(), rtol=1e-4, atol=1e-6)
    checked = 0
    for n, prm in dec.named_parameters():
        if pr[n].grad is None:
            continue
        gref = pr[n].grad
        if n == "embedding.weight":  # nn.Embedding(padding_idx=pad): the pad row gets no gradient
            gref[pad] = 0
        torch.testing.assert_close(prm._capk_grad.cpu(), gref, rtol=2e-3, atol=2e-3 * float(gref.abs().max()) + 1e-8,
                                   msg=lambda m: f"{n}: {m}")
        checked += 1
    assert checked >= 8


# --------------------------------------------------------------------- CLI train ----
@cuda
def test_cli_main_train_steps_and_checkpoint(tmp_path):
    """capk.main (src/main.py:17-102) --mode train on the config-3 model (ViT-B/16 +
    Transformer decoder, bf16) for 2 synthetic batches at batch 8 -- 2 CE steps, then (the
    reference default use_rl=True) 2 SCST updates over the same batches -- then save / load
    a checkpoint through the trainer (trainer.py:569-620 layout)."""
    from capk.main import main
    cfg, model, trainer = main(["--mode", "train", "--encoder_type", "vit", "--decoder_type", "transformer",
                                "--attention_type", "multi_head", "--batch_size", "8", "--steps", "2",
                                "--output_dir", str(tmp_path), "--seed", "3"])
    assert trainer is not None and trainer.global_step == 4 and trainer.rl_updates == 2
    path = trainer.save_checkpoint(0, path=os.path.join(str(tmp_path), "ck.pth"))
    before = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    trainer.train_step(*_batch(cfg))  # move the weights, then restore them from the file
    trainer.load_checkpoint(path)
    after = model.state_dict()
    for k, v in before.items():
        assert torch.equal(after[k].cpu(), v), k
    assert trainer.global_step == 4 and trainer.rl_updates == 2


def _batch(cfg):
    g = torch.Generator(device="cuda").manual_seed(9)
    images = torch.randn(8, 3, 224, 224, device="cuda", generator=g)
    caps = torch.randint(0, cfg.model.pad_token_id, (8, 20), device="cuda", generator=g)
    return images, caps
