"""Config-4 path on the GPU: CLIP-ViT encoder (A2) + GPT-2 decoder with the D7 image
prefix (A12), and GPT-2 beam search (A14).

* fp32 vs tests/golden/clip_gpt2_step.npz (the reference's own forward / CombinedLoss /
  backward, oracle/gen_golden.py): encoder features + pooled, logits, loss and every
  parameter gradient; image_prefix / visual_projection get no gradient (unused).
* bf16 step: logits within 3e-2 relative of the fp32 golden logits.
* GPT-2 beam-5 (KV cache with the 10 prefix rows) vs oracle/beam.py over the oracle
  GPT-2 re-run on each prefix: sequences and beam indices bit-exact.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "clip_gpt2_step.npz")


def _model(precision):
    import capk
    from capk import config as C
    from capk.models import captioning_model as cm
    from capk.models import encoders as E
    z = np.load(GOLD, allow_pickle=False)
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in z["meta/dims"]]
    cfg = C.Config()
    cfg.model.encoder = C.EncoderConfig(encoder_type="clip", pretrained_model_name="capk-test-tiny", feature_dim=D)
    cfg.model.decoder = C.DecoderConfig(decoder_type="gpt2", pretrained_model_name=None, hidden_dim=D, num_layers=Ld,
                                        num_heads=Hd, max_length=40)
    cfg.model.vocab_size, cfg.model.pad_token_id = V, pad
    cfg.model.bos_token_id = cfg.model.eos_token_id = pad
    E.CLIP_ARCHS["capk-test-tiny"] = dict(hidden_size=D, num_hidden_layers=Le, num_attention_heads=He,
                                          intermediate_size=2 * D, image_size=img, patch_size=patch, num_channels=3,
                                          layer_norm_eps=1e-5)
    model = cm.ImageCaptioningModel(cfg)
    sd = {k[3:]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("p0/")}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected and missing == ["decoder.model.lm_head.weight"], (missing, unexpected)  # tied to wte
    store = capk.prepare(model, "cuda", precision)
    model.eval()
    return z, model, store, cfg


@cuda
def test_clip_gpt2_golden_step_fp32():
    from capk.train import CombinedLoss
    z, model, store, cfg = _model("fp32")
    images = torch.from_numpy(z["in/images"]).cuda()
    caps = torch.from_numpy(z["in/captions"]).cuda()
    enc = model.encoder(images)
    np.testing.assert_allclose(enc["features"].detach().cpu().numpy(), z["out/features"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(enc["pooled_features"].detach().cpu().numpy(), z["out/pooled"], rtol=1e-4, atol=1e-5)
    out = model(images=images, captions=caps)
    np.testing.assert_allclose(out["logits"].detach().cpu().numpy(), z["out/logits"], rtol=1e-4, atol=1e-5)
    loss = CombinedLoss(cfg.model.pad_token_id)(logits=out["logits"], targets=caps)["total_loss"]
    np.testing.assert_allclose(float(loss), float(z["out/loss"][0]), rtol=1e-5)
    loss.backward()
    names = dict(model.named_parameters())
    for n, p in names.items():
        key = "grad/" + n
        g = p._capk_grad.detach().cpu().numpy()
        if key in z.files:
            ref = z[key]
            tol = 2e-4 * float(np.abs(ref).max()) + 1e-7
            np.testing.assert_allclose(g, ref, rtol=2e-4, atol=tol, err_msg=n)
        else:
            assert n in ("decoder.image_prefix", "decoder.visual_projection.weight",
                         "decoder.visual_projection.bias"), n


@cuda
def test_clip_gpt2_bf16_logits_close():
    z, model, store, cfg = _model("bf16")
    images = torch.from_numpy(z["in/images"]).cuda()
    caps = torch.from_numpy(z["in/captions"]).cuda()
    with torch.no_grad():
        got = model(images=images, captions=caps)["logits"].float().cpu()
    ref = torch.from_numpy(z["out/logits"])
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 3e-2, rel


@cuda
def test_clip_gpt2_bf16_train_steps_reduce_loss():
    from capk.train import CapkAdamW, CombinedLoss
    z, model, store, cfg = _model("bf16")
    model.train()  # dropout 0.1 at the embedding, attention and both residual sites
    images = torch.from_numpy(z["in/images"]).cuda()
    caps = torch.from_numpy(z["in/captions"]).cuda()
    opt = CapkAdamW(store, lr=3e-3, weight_decay=0.01)
    lf = CombinedLoss(cfg.model.pad_token_id)
    losses = []
    for _ in range(8):
        loss = lf(logits=model(images=images, captions=caps)["logits"], targets=caps)["total_loss"]
        loss.backward()
        opt.step(lr=3e-3)
        losses.append(float(loss))
    assert all(np.isfinite(losses)) and losses[-1] < losses[0] * 0.9, losses
    # unused parameters never move (AdamW skips grad-less parameters)
    p0 = torch.from_numpy(z["p0/decoder.image_prefix"])
    assert torch.equal(model.decoder.image_prefix.detach().cpu(), p0)


@cuda
def test_gpt2_beam5_vs_oracle_fp32():
    from oracle import decoders as odec
    from oracle import encoders as oenc
    from oracle.beam import beam_search as oracle_beam
    z, model, store, cfg = _model("fp32")
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in z["meta/dims"]]
    images = torch.from_numpy(z["in/images"])
    with torch.no_grad():
        ids, info = model.generate(images=images.cuda(), max_length=12, num_beams=5)
    sd = {k: v.detach().cpu().float() for k, v in model.state_dict().items()}
    enc = oenc.clip_encoder({k[len("encoder.model."):]: v for k, v in sd.items() if k.startswith("encoder.model.")},
                            images, Le, He, patch)
    p = {k[len("decoder."):]: v for k, v in sd.items() if k.startswith("decoder.")}
    pooled = enc["pooled_features"].repeat_interleave(5, 0)

    def fn(seqs):
        with torch.no_grad():
            return odec.gpt2_decoder(p, pooled, seqs, Ld, Hd, pad, use_pad_mask=False)[:, -1]

    ref = oracle_beam(fn, images.shape[0], 5, 12, bos=pad, eos=pad, pad=pad)
    assert torch.equal(ids.cpu(), ref["sequences"])
    assert torch.equal(info["beam_indices"].cpu(), ref["beam_indices"])
    torch.testing.assert_close(info["sequences_scores"].cpu(), ref["sequences_scores"], rtol=1e-4, atol=1e-5)


@cuda
def test_gpt2_scst_sampling_and_update_vs_oracle():
    """Config-5 RL step (A16 on A12): the KV-cached GPT-2 sampler (D7 prefix) vs the oracle
    sampler (oracle/scst.py) over the oracle GPT-2 re-run on each prefix (trainer.py:383-438
    semantics: generate()'s all-ones mask); then one SCST update with the reference's GPT-2
    baseline (beam-4 generate, trainer.py:353-356 -> decoders.py:645-654): the loss and every
    decoder gradient vs torch autograd of the oracle decoder."""
    import torch.nn.functional as F
    from capk.train import CapkAdamW
    from capk.train.scst import cider_d, pg_targets, sample_captions, scst_step, strip_special
    from oracle import decoders as odec
    from oracle import encoders as oenc
    from oracle import scst as oscst
    z, model, store, cfg = _model("fp32")
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in z["meta/dims"]]
    images = torch.from_numpy(z["in/images"]).cuda()
    B = images.shape[0]
    seed, L = 91, 9
    sd = {k: v.detach().cpu().float().clone() for k, v in model.state_dict().items()}
    with torch.no_grad():
        enc = model.encoder(images)
        ids, logp = sample_captions(model.decoder, enc, L, seed=seed)
    p = {k[len("decoder."):]: v for k, v in sd.items() if k.startswith("decoder.")}
    with torch.no_grad():
        pooled = oenc.clip_encoder({k[len("encoder.model."):]: v for k, v in sd.items()
                                    if k.startswith("encoder.model.")}, images.cpu(), Le, He, patch)["pooled_features"]
        oids = torch.full((B, 1), pad, dtype=torch.long)
        olp = []
        for t in range(L - 1):
            lg = odec.gpt2_decoder(p, pooled, oids, Ld, Hd, pad, use_pad_mask=False)[:, -1]
            picks = [oscst.sample_row(lg[r].numpy(), seed, t, r) for r in range(B)]
            nxt = torch.tensor([tok for tok, _, _ in picks])
            olp.append([lp for _, lp, _ in picks])
            oids = torch.cat([oids, nxt[:, None]], 1)
            if bool((nxt == pad).all()):
                break
    assert torch.equal(ids.cpu(), oids), (ids.cpu(), oids)
    np.testing.assert_allclose(logp.cpu().numpy(), np.array(olp, dtype=np.float32).T, rtol=1e-4, atol=1e-4)
    # one SCST update with the beam-4 baseline
    refs = [[[3, 5, 7, 9], [5, 7]], [[1, 2, 3]], [[4, 4, 8, 15, 16]]][:B]
    while len(refs) < B:
        refs.append([[2, 4, 6]])
    opt = CapkAdamW(store, lr=0.0, weight_decay=0.0)
    loss, rs, rb = scst_step(model, images, refs, opt, lr=0.0, seed=seed, max_length=L,
                             baseline_kwargs={"num_beams": 4})
    samp = [strip_special(r, pad, pad, pad) for r in ids.cpu().tolist()]
    with torch.no_grad():
        base_ids, _ = model.decoder.generate({"pooled_features": enc["pooled_features"]}, L, num_beams=4)
    base = [strip_special(r, pad, pad, pad) for r in base_ids.cpu().tolist()]
    adv = torch.tensor(cider_d(samp, refs) - cider_d(base, refs), dtype=torch.float32)
    assert abs(float(adv.abs().sum())) > 0  # a non-trivial advantage exercises the gradient
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    logits = odec.gpt2_decoder(pr, pooled, ids.cpu(), Ld, Hd, pad, use_pad_mask=False)
    tgt = pg_targets(ids.cpu(), pad)
    lp = F.log_softmax(logits[:, :-1], -1).gather(-1, tgt[:, 1:].clamp(min=0)[..., None])[..., 0]
    mask = (tgt[:, 1:] != -100).float()
    ref = -(lp * adv[:, None] * mask).sum() / mask.sum()
    ref.backward()
    torch.testing.assert_close(loss.cpu(), ref.detach(), rtol=1e-4, atol=1e-6)
    checked = 0
    for n, prm in model.decoder.named_parameters():
        if pr[n].grad is None:
            continue
        gref = pr[n].grad
        torch.testing.assert_close(prm._capk_grad.cpu(), gref, rtol=2e-3, atol=2e-3 * float(gref.abs().max()) + 1e-8,
                                   msg=lambda m: f"{n}: {m}")
        checked += 1
    assert checked >= 4 * Ld
