"""Legacy Show-Attend-Tell path (config 1) on the GPU vs the reference's own
step (tests/golden/legacy_decoder_step.npz, oracle/gen_golden.py): predictions, alphas,
loss (packed CE + attention regulariser), d(encoder_out), every parameter gradient and
the clamped-Adam update (fp32; digests for the large tensors).  The legacy encoder
(torchvision resnet101 trunk + AdaptiveAvgPool2d(14)) vs the CPU oracle under the
torchvision->HF name mapping (torchvision itself is not installed: parity vs torchvision
unpinned, architecture identical).  bf16 train steps reduce the loss."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "legacy_decoder_step.npz")


def _rel(a, b):
    b = b.to(a.device)
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


def _check_digest(z, key, t, rtol, atol_frac):
    a = t.detach().double().cpu().numpy()
    if key in z.files:
        ref = z[key]
        np.testing.assert_allclose(a, ref, rtol=rtol, atol=atol_frac * float(np.abs(ref).max()) + 1e-12, err_msg=key)
        return
    head, stats = z[key + "@head"], z[key + "@stats"]
    flat = a.reshape(-1)
    np.testing.assert_allclose(flat[:head.size], head, rtol=rtol, atol=atol_frac * float(np.abs(head).max()) + 1e-12,
                               err_msg=key)
    got = np.array([flat.sum(), np.abs(flat).sum(), np.sqrt((flat * flat).sum())])
    np.testing.assert_allclose(got[1:], stats[1:], rtol=max(rtol, 1e-6), err_msg=key + " stats")
    assert abs(got[0] - stats[0]) <= max(rtol, 1e-6) * stats[1] + 1e-12, (key, got[0], stats[0])


def _check_digest_abs(z, key, t, atol):
    a = t.detach().double().cpu().numpy()
    if key in z.files:
        np.testing.assert_allclose(a, z[key], rtol=0, atol=atol, err_msg=key)
        return
    head, stats = z[key + "@head"], z[key + "@stats"]
    flat = a.reshape(-1)
    np.testing.assert_allclose(flat[:head.size], head, rtol=0, atol=atol, err_msg=key)
    assert abs(flat.sum() - stats[0]) <= atol * flat.size, key


def _decoder(precision, V=40, seed=2024):
    import capk
    from capk.legacy import Decoder
    torch.manual_seed(seed)
    dec = Decoder(V, False, "cuda")
    store = capk.prepare(dec, "cuda", precision)
    return dec, store


@cuda
def test_legacy_decoder_golden_fp32():
    from capk.legacy import LegacyAdam, LegacyCaptionLoss
    z = np.load(GOLD, allow_pickle=False)
    dec, store = _decoder("fp32")
    for n, p in dec.named_parameters():
        _check_digest(z, "p0/" + n, p, 0, 0)
    dec.train()
    dec.dropout.p = 0.0  # the golden step ran with dropout off
    enc = torch.from_numpy(z["in/encoder_out"]).cuda().requires_grad_(True)
    caps = torch.from_numpy(z["in/captions"]).cuda()
    lengths = [int(x) for x in z["in/lengths"]]
    preds, caps_sorted, dec_len, alphas = dec(enc, caps, lengths)
    assert dec_len == [x - 1 for x in lengths]
    np.testing.assert_allclose(preds.detach().cpu().numpy(), z["out/predictions"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(alphas.detach().cpu().numpy(), z["out/alphas"], rtol=1e-4, atol=1e-7)
    loss = LegacyCaptionLoss()(preds, alphas, caps_sorted, dec_len)
    np.testing.assert_allclose(float(loss.detach()), float(z["out/loss"][0]), rtol=1e-5)
    opt = LegacyAdam(store, lr=4e-4)
    opt.zero_grad()
    loss.backward()
    torch.cuda.synchronize()
    ref = z["out/dencoder_out"]
    np.testing.assert_allclose(enc.grad.cpu().numpy(), ref, rtol=1e-4, atol=1e-4 * float(np.abs(ref).max()))
    # att.bias: softmax is shift-invariant, its gradient is analytically 0 (both sides are
    # fp32 noise), so Adam's first step moves it by at most lr in either direction
    zero_grad = {"att.bias"}
    p0 = {n: p.detach().clone() for n, p in dec.named_parameters()}
    for n, p in dec.named_parameters():
        if n in zero_grad:
            assert float(p._capk_grad.abs().max()) < 1e-6 and float(np.abs(z["grad/" + n]).max()) < 1e-6
            continue
        _check_digest(z, "grad/" + n, p._capk_grad, 2e-4, 2e-4)
    g0 = {n: p._capk_grad.detach().clone() for n, p in dec.named_parameters()}
    opt.step()
    torch.cuda.synchronize()
    for n, p in dec.named_parameters():
        # (a) the fused clamp + Adam kernel is exactly torch Adam's first step on our gradient
        g = g0[n].double().clamp(-5, 5)
        want = p0[n].double() - 4e-4 * g / (g.abs() + 1e-8)
        assert float((p.detach().double() - want).abs().max()) < 1e-8, n
        if n in zero_grad:
            assert float((p.detach() - p0[n]).abs().max()) <= 4e-4 * (1 + 1e-5)
            continue
        # (b) vs the reference's update: Adam's first step is lr * g / (|g| + eps), so
        # elements whose gradient is near eps amplify fp32 gradient noise: 1% of lr
        _check_digest_abs(z, "p1/" + n, p, 4e-6)


@cuda
def test_legacy_decoder_ragged_batch_and_no_encoder_grad():
    """Shrinking batch with equal and distinct lengths; encoder_out without grad (train.py's
    decoder-only optimizer); predictions are zero past each caption's decode length."""
    from capk.legacy import LegacyCaptionLoss
    dec, _ = _decoder("fp32", V=64, seed=3)
    dec.train()
    enc = torch.randn(5, 7, 7, 2048, device="cuda")
    lengths = [9, 9, 6, 3, 2]
    caps = torch.randint(3, 64, (5, 9), device="cuda")
    preds, _, dec_len, alphas = dec(enc, caps, lengths)
    for b, d in enumerate(dec_len):
        assert not preds[b, d:].any() and not alphas[b, d:].any()
        assert torch.allclose(alphas[b, :d].sum(-1), torch.ones(d, device="cuda"), atol=1e-5)
    loss = LegacyCaptionLoss()(preds, alphas, caps, dec_len)
    loss.backward()
    assert torch.isfinite(loss)
    with pytest.raises(RuntimeError):
        LegacyCaptionLoss()(preds, alphas, caps, [1, 3, 2, 2, 1])


def _tv_to_hf(sd):
    """torchvision resnet trunk names (models/encoder.py Sequential) -> transformers ResNetModel names."""
    out = {}
    for k, v in sd.items():
        parts = k.split(".")
        if parts[1] == "0":
            out["embedder.embedder.convolution." + parts[2]] = v
        elif parts[1] == "1":
            out["embedder.embedder.normalization." + parts[2]] = v
        else:
            si, li, name = int(parts[1]) - 4, parts[2], parts[3]
            pre = f"encoder.stages.{si}.layers.{li}."
            if name.startswith("conv"):
                out[pre + f"layer.{int(name[4:]) - 1}.convolution." + parts[4]] = v
            elif name.startswith("bn"):
                out[pre + f"layer.{int(name[2:]) - 1}.normalization." + parts[4]] = v
            else:  # downsample.{0,1}
                sub = "convolution." if parts[4] == "0" else "normalization."
                out[pre + "shortcut." + sub + parts[5]] = v
    return out


@cuda
def test_legacy_encoder_vs_oracle_fp32():
    import capk
    from capk.legacy import Encoder
    from oracle import encoders as oenc
    torch.manual_seed(9)
    enc = Encoder(layers=(1, 2, 1, 1))
    sd = {k: v.detach().clone() for k, v in enc.state_dict().items()}
    capk.prepare(enc, "cuda", "fp32")
    enc.train()
    images = torch.randn(2, 3, 64, 64)
    with torch.no_grad():
        out = enc(images.cuda())
        hf = _tv_to_hf(sd)
        last, _ = oenc.resnet_model(hf, images, [256, 512, 1024, 2048], [1, 2, 1, 1], training=True,
                                    state={k: v.clone() for k, v in hf.items()})
        ref = F.adaptive_avg_pool2d(last, (14, 14)).permute(0, 2, 3, 1)
    assert out.shape == (2, 14, 14, 2048)
    assert _rel(out, ref) < 1e-4


@cuda
def test_legacy_train_steps_bf16_reduce_loss():
    import capk
    from capk.legacy import Encoder, LegacyAdam, LegacyCaptionLoss, train_step
    torch.manual_seed(1)
    enc = Encoder(layers=(1, 1, 1, 1))
    capk.prepare(enc, "cuda", "bf16")
    dec, store = _decoder("bf16", V=128, seed=4)
    enc.train()
    dec.train()
    opt = LegacyAdam(store, lr=4e-4)
    crit = LegacyCaptionLoss()
    imgs = torch.randn(4, 3, 96, 96, device="cuda")
    lengths = [12, 10, 10, 7]
    caps = torch.randint(3, 128, (4, 12), device="cuda")
    losses = [float(train_step(enc, dec, opt, crit, imgs, caps, lengths).detach()) for _ in range(8)]
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses
