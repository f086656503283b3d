"""Pin the CPU oracle against golden vectors produced by the reference itself.

The fixtures in tests/golden/ were written by oracle/gen_golden.py, which runs
the reference's own ImageCaptioningModel / TransformerDecoder / CombinedLoss /
CaptioningTrainer._create_optimizer code (build container only).  These tests
run anywhere (CPU) and never touch /root/reference.
"""
import os

import numpy as np
import pytest
import torch

from oracle import decoders as odec
from oracle import encoders as oenc
from oracle import train as otrain


def _load(golden_dir, name):
    path = os.path.join(golden_dir, name + ".npz")
    return np.load(path, allow_pickle=False)


def _params(z, tag):
    out = {}
    for k in z.files:
        if k.startswith(tag + "/"):
            out[k[len(tag) + 1:]] = torch.from_numpy(z[k].copy())
    return out


def _sub(p, prefix):
    return {k[len(prefix):]: v for k, v in p.items() if k.startswith(prefix)}


def _forward(p, z):
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in z["meta/dims"]]
    images = torch.from_numpy(z["in/images"])
    caps = torch.from_numpy(z["in/captions"])
    enc = oenc.vit_encoder(_sub(p, "encoder.model."), images, Le, He, patch)
    logits = odec.transformer_decoder(_sub(p, "decoder."), enc["features"], caps, Ld, Hd, pad)
    loss = otrain.shifted_ce(logits, caps, pad)
    return enc, logits, loss


@pytest.fixture(scope="module")
def vt(golden_dir):
    return _load(golden_dir, "vit_transformer_step")


def test_vit_transformer_forward_matches_reference(vt):
    p = _params(vt, "p0")
    enc, logits, loss = _forward(p, vt)
    np.testing.assert_allclose(enc["features"].detach().numpy(), vt["out/features"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(enc["pooled_features"].detach().numpy(), vt["out/pooled"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(logits.detach().numpy(), vt["out/logits"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(loss.item(), vt["out/loss"][0], rtol=1e-6)


def test_vit_transformer_grads_match_reference(vt):
    p = {k: v.requires_grad_(True) for k, v in _params(vt, "p0").items()}
    _, _, loss = _forward(p, vt)
    loss.backward()
    ref = _params(vt, "grad")
    for n, t in p.items():
        if n in ref:
            assert t.grad is not None, n
            np.testing.assert_allclose(t.grad.numpy(), ref[n].numpy(), rtol=1e-4, atol=1e-6, err_msg=n)
        else:  # reference had grad None (e.g. ViT pooler: pooled unused by this decoder)
            assert t.grad is None or float(t.grad.abs().max()) == 0.0, n


def test_adamw_groups_and_schedule_match_reference(vt):
    p0, p1, p2, g = _params(vt, "p0"), _params(vt, "p1"), _params(vt, "p2"), _params(vt, "grad")
    lrs = vt["out/lrs"]
    for step, lr in enumerate(lrs):
        np.testing.assert_allclose(otrain.cosine_warmup_lr(step, 5e-3, 2, 10), lr, rtol=1e-12)
    ref_nd = set(str(s) for s in vt["opt/no_decay"])
    for n in p0:
        assert otrain.no_decay(n) == (n in ref_nd), n
    for n in p0:
        if n not in g:  # no grad -> AdamW skips the parameter
            np.testing.assert_array_equal(p1[n].numpy(), p0[n].numpy())
            continue
        wd = 0.0 if otrain.no_decay(n) else 0.01
        p, m, v = p0[n].clone(), torch.zeros_like(p0[n]), torch.zeros_like(p0[n])
        otrain.adamw_step(p, g[n], m, v, 1, lrs[0], wd)
        np.testing.assert_allclose(p.numpy(), p1[n].numpy(), rtol=1e-6, atol=1e-7, err_msg=n)
        otrain.adamw_step(p, g[n], m, v, 2, lrs[1], wd)
        np.testing.assert_allclose(p.numpy(), p2[n].numpy(), rtol=1e-6, atol=1e-7, err_msg=n)


def test_greedy_generate_matches_reference(vt):
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in vt["meta/dims"]]
    p = _params(vt, "p0")
    images = torch.from_numpy(vt["in/images"])
    with torch.no_grad():
        enc = oenc.vit_encoder(_sub(p, "encoder.model."), images, Le, He, patch)
        ids = odec.transformer_greedy(_sub(p, "decoder."), enc["features"], 6, Ld, Hd, pad, pad)
    np.testing.assert_array_equal(ids.numpy(), vt["out/greedy_ids"])


# ------------------------------------------------ config 4: CLIP + GPT-2 (D7) --
@pytest.fixture(scope="module")
def cg(golden_dir):
    return _load(golden_dir, "clip_gpt2_step")


def _forward_cg(p, z):
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in z["meta/dims"]]
    images = torch.from_numpy(z["in/images"])
    caps = torch.from_numpy(z["in/captions"])
    enc = oenc.clip_encoder(_sub(p, "encoder.model."), images, Le, He, patch)
    logits = odec.gpt2_decoder(_sub(p, "decoder."), enc["pooled_features"], caps, Ld, Hd, pad)
    return enc, logits, otrain.shifted_ce(logits, caps, pad)


def test_clip_gpt2_forward_matches_reference(cg):
    enc, logits, loss = _forward_cg(_params(cg, "p0"), cg)
    np.testing.assert_allclose(enc["features"].detach().numpy(), cg["out/features"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(enc["pooled_features"].detach().numpy(), cg["out/pooled"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(logits.detach().numpy(), cg["out/logits"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(loss.item(), cg["out/loss"][0], rtol=1e-6)


def test_clip_gpt2_grads_match_reference(cg):
    p = {k: v.requires_grad_(True) for k, v in _params(cg, "p0").items()}
    _, _, loss = _forward_cg(p, cg)
    loss.backward()
    ref = _params(cg, "grad")
    for n, t in p.items():
        if n in ref:
            assert t.grad is not None, n
            np.testing.assert_allclose(t.grad.numpy(), ref[n].numpy(), rtol=1e-4, atol=1e-6, err_msg=n)
        else:  # image_prefix / visual_projection: unused by the reference forward (grad None)
            assert t.grad is None or float(t.grad.abs().max()) == 0.0, n


# ------------------------------------------- LSTM decoder + attention types --
LSTM_VARIANTS = [("soft", "soft", 1, 0.7), ("multi_head", "multi_head", 4, 1.0), ("aoa", "aoa", 4, 1.0),
                 ("adaptive", "adaptive", 4, 1.0), ("adaptive_soft", "adaptive", 1, 1.0)]


@pytest.mark.parametrize("name,kind,heads,temp", LSTM_VARIANTS)
def test_lstm_attention_matches_reference(golden_dir, name, kind, heads, temp):
    from oracle import lstm as olstm
    z = _load(golden_dir, "lstm_attention")
    D, L, V, B, T, S, pad = [int(x) for x in z["meta/dims"]]
    p = {k[len(name) + 4:]: torch.from_numpy(z[k].copy()).requires_grad_(True) for k in z.files
         if k.startswith(name + "/p0/")}
    feats = torch.from_numpy(z["in/features"]).requires_grad_(True)
    pooled = torch.from_numpy(z["in/pooled"]).requires_grad_(True)
    caps = torch.from_numpy(z["in/captions"])
    logits, w = olstm.lstm_decoder(p, feats, pooled, caps, L, kind, heads, temp)
    np.testing.assert_allclose(logits.detach().numpy(), z[name + "/logits"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(w.detach().numpy(), z[name + "/attention_weights"], rtol=1e-5, atol=1e-6)
    loss = otrain.shifted_ce(logits, caps, pad)
    np.testing.assert_allclose(loss.item(), z[name + "/loss"][0], rtol=1e-6)
    loss.backward()
    np.testing.assert_allclose(feats.grad.numpy(), z[name + "/dfeatures"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(pooled.grad.numpy(), z[name + "/dpooled"], rtol=1e-4, atol=1e-7)
    for n, t in p.items():
        key = name + "/grad/" + n
        if key in z.files:
            np.testing.assert_allclose(t.grad.numpy(), z[key], rtol=1e-4, atol=1e-7, err_msg=n)
        else:
            assert t.grad is None or float(t.grad.abs().max()) == 0.0, n
    with torch.no_grad():
        ids = olstm.lstm_greedy({k: v.detach() for k, v in p.items()}, feats.detach(), pooled.detach(), 6, L, kind,
                                pad, heads, temp)
    np.testing.assert_array_equal(ids.numpy(), z[name + "/greedy_ids"])


# ------------------------------------------------------------ config 2 (A3 + A6/A7) --
RESNET_TINY = dict(hidden_sizes=[32, 64, 64, 128], depths=[2, 1, 2, 1])


def test_resnet_lstm_step_matches_reference(golden_dir):
    """Oracle ResNet (train-mode BN) + LSTM/soft decoder vs the reference's own step:
    logits, loss, every gradient, running buffers after two passes, eval-mode features."""
    from oracle import lstm as olstm
    z = _load(golden_dir, "resnet_lstm_step")
    D, L, V, B, T, pad, img = [int(x) for x in z["meta/dims"]]
    s0 = _params(z, "s0")
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in s0.items()}
    images = torch.from_numpy(z["in/images"])
    caps = torch.from_numpy(z["in/captions"])
    state = {k: v.clone() for k, v in s0.items()}
    enc = oenc.resnet_encoder(_sub(p, "encoder."), images, training=True, state=_sub(state, "encoder."),
                              **RESNET_TINY)
    logits, _ = olstm.lstm_decoder(_sub(p, "decoder."), enc["features"], enc["pooled_features"], caps, L, "soft")
    np.testing.assert_allclose(logits.detach().numpy(), z["out/logits"], rtol=1e-4, atol=1e-5)
    loss = otrain.shifted_ce(logits, caps, pad)
    np.testing.assert_allclose(float(loss), float(z["out/loss"][0]), rtol=1e-5)
    loss.backward()
    for n, t in p.items():
        if "grad/" + n in z.files:
            ref = z["grad/" + n]
            np.testing.assert_allclose(t.grad.numpy(), ref, rtol=1e-4, atol=1e-4 * float(np.abs(ref).max()) + 1e-9,
                                       err_msg=n)
    with torch.no_grad():
        ftr = oenc.resnet_encoder(_sub(p, "encoder."), images, training=True, state=_sub(state, "encoder."),
                                  **RESNET_TINY)
        np.testing.assert_allclose(ftr["features"].numpy(), z["out/features_train"], rtol=1e-4, atol=1e-5)
        for k in z.files:
            if k.startswith("s2/") and "running" in k:
                np.testing.assert_allclose(state[k[3:]].numpy(), z[k], rtol=1e-5, atol=1e-6, err_msg=k)
        fev = oenc.resnet_encoder(_sub(p, "encoder."), images, training=False, state=_sub(state, "encoder."),
                                  **RESNET_TINY)
        np.testing.assert_allclose(fev["features"].numpy(), z["out/features_eval"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(fev["pooled_features"].numpy(), z["out/pooled_eval"], rtol=1e-4, atol=1e-5)


# ------------------------------------------------------------ config 1 (A11) --
def _check_digest(z, key, t, rtol, atol_frac):
    a = t.detach().double().numpy()
    if key in z.files:
        ref = z[key]
        np.testing.assert_allclose(a, ref, rtol=rtol, atol=atol_frac * float(np.abs(ref).max()) + 1e-12, err_msg=key)
        return
    head, stats = z[key + "@head"], z[key + "@stats"]
    flat = a.reshape(-1)
    np.testing.assert_allclose(flat[:head.size], head, rtol=rtol, atol=atol_frac * float(np.abs(head).max()) + 1e-12,
                               err_msg=key)
    got = np.array([flat.sum(), np.abs(flat).sum(), np.sqrt((flat * flat).sum())])
    np.testing.assert_allclose(got[1:], stats[1:], rtol=rtol, err_msg=key + " stats")
    assert abs(got[0] - stats[0]) <= rtol * stats[1] + 1e-12, (key, got[0], stats[0])


def legacy_params_from_seed():
    """The build's legacy Decoder created under the golden's seed (same module/RNG order as
    models/decoder.py:9-58) -> the reference's initial parameters (pinned by digests)."""
    from capk.legacy import Decoder
    torch.manual_seed(2024)
    return {n: p.detach().clone() for n, p in Decoder(40, False, "cpu").named_parameters()}


def test_legacy_decoder_step_matches_reference(golden_dir):
    from oracle import legacy as oleg
    z = _load(golden_dir, "legacy_decoder_step")
    p0 = legacy_params_from_seed()
    for n, t in p0.items():
        _check_digest(z, "p0/" + n, t, 0, 0)
    p = {n: t.clone().requires_grad_(True) for n, t in p0.items()}
    enc = torch.from_numpy(z["in/encoder_out"]).requires_grad_(True)
    caps = torch.from_numpy(z["in/captions"])
    lengths = [int(x) for x in z["in/lengths"]]
    preds, alphas = oleg.legacy_decoder(p, enc, caps, lengths)
    np.testing.assert_allclose(preds.detach().numpy(), z["out/predictions"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(alphas.detach().numpy(), z["out/alphas"], rtol=1e-4, atol=1e-7)
    loss = oleg.legacy_loss(preds, alphas, caps, lengths)
    np.testing.assert_allclose(float(loss), float(z["out/loss"][0]), rtol=1e-5)
    loss.backward()
    np.testing.assert_allclose(enc.grad.numpy(), z["out/dencoder_out"], rtol=1e-4,
                               atol=1e-4 * float(np.abs(z["out/dencoder_out"]).max()))
    for n, t in p.items():
        _check_digest(z, "grad/" + n, t.grad, 1e-4, 1e-4)
    p1 = oleg.clamp_adam_step({n: t.detach() for n, t in p.items()}, {n: t.grad for n, t in p.items()})
    for n, t in p1.items():
        _check_digest(z, "p1/" + n, t, 1e-5, 1e-6)


def test_qformer_matches_reference(golden_dir):
    """oracle/encoders.py qformer vs the reference QFormer (captioning_model.py:153-245):
    queries and every parameter / feature gradient (eval mode)."""
    z = _load(golden_dir, "qformer_step")
    D, Q, H, S, B = [int(x) for x in z["meta/dims"]]
    p = {k: v.requires_grad_(True) for k, v in _params(z, "p0").items()}
    feats = torch.from_numpy(z["in/features"]).requires_grad_(True)
    out = oenc.qformer(p, feats, 2, H)
    np.testing.assert_allclose(out.detach().numpy(), z["out/queries"], rtol=1e-5, atol=1e-6)
    (out * torch.from_numpy(z["in/grad_out"])).sum().backward()
    np.testing.assert_allclose(feats.grad.numpy(), z["out/dfeatures"], rtol=1e-4, atol=1e-6)
    for n, t in p.items():
        ref = z["grad/" + n]
        np.testing.assert_allclose(t.grad.numpy(), ref, rtol=1e-4, atol=1e-6 * max(1.0, float(np.abs(ref).max())),
                                   err_msg=n)


def test_swin_encoder_matches_reference(golden_dir):
    """oracle/encoders.py swin_encoder vs the reference SwinEncoder.forward
    (src/models/encoders.py:140-182 on transformers SwinModel, oracle/gen_golden.py
    case_swin_encoder): features, pooled and every parameter gradient.  The k_proj bias
    gradients are exactly zero in exact arithmetic (softmax is invariant to a per-query
    shift), so they are compared against an absolute floor."""
    z = _load(golden_dir, "swin_encoder")
    depths = [int(x) for x in z["meta/depths"]]
    heads = [int(x) for x in z["meta/heads"]]
    p = {k: v.requires_grad_(True) for k, v in _params(z, "p0").items()}
    f, pooled = oenc.swin_encoder(p, torch.from_numpy(z["in/images"]), depths, heads)
    np.testing.assert_allclose(f.detach().numpy(), z["out/features"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(pooled.detach().numpy(), z["out/pooled"], rtol=1e-5, atol=1e-6)
    ((f * torch.from_numpy(z["in/gf"])).sum() + (pooled * torch.from_numpy(z["in/gp"])).sum()).backward()
    for n, t in p.items():
        ref = z["grad/" + n]
        np.testing.assert_allclose(t.grad.numpy(), ref, rtol=1e-4, atol=1e-6 * max(1.0, float(np.abs(ref).max())),
                                   err_msg=n)


def test_swin_state_dict_names_match_reference(golden_dir):
    """capk's SwinEncoder exposes the reference SwinEncoder's state-dict names (model.* of
    transformers SwinModel + proj.*), so a reference checkpoint loads unchanged."""
    from capk import config as C
    from capk.models.encoders import SwinEncoder
    z = _load(golden_dir, "swin_encoder")
    img, P, E, ws, Fd, B = [int(x) for x in z["meta/dims"]]
    arch = dict(image_size=img, patch_size=P, num_channels=3, embed_dim=E, depths=tuple(int(x) for x in z["meta/depths"]),
                num_heads=tuple(int(x) for x in z["meta/heads"]), window_size=ws, mlp_ratio=4.0, qkv_bias=True,
                layer_norm_eps=1e-5, drop_path_rate=0.1)
    enc = SwinEncoder(C.EncoderConfig(encoder_type="swin", feature_dim=Fd), arch=arch)
    want = {k[3:]: z[k].shape for k in z.files if k.startswith("p0/")}
    got = {k: tuple(v.shape) for k, v in enc.state_dict().items()}
    assert got == want
