"""SCST (A16) on the GPU: the Categorical sampler kernel vs oracle/scst.py, the weighted
(policy-gradient) CE kernel vs a PyTorch fp32 reference, sampled sequences of the tiny
golden Transformer model vs the oracle sampler over the oracle decoder, and a full SCST
update (loss and every decoder gradient vs torch autograd of the oracle)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import scst as oscst

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@cuda
@pytest.mark.parametrize("V,scale", [(50257, 3.0), (61, 1.0)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sample_rows_vs_oracle(V, scale, dtype):
    """fp32 rows: the chunk-owner kernel; bf16 rows: the LDS-staged kernel (same arithmetic
    on the bf16 values, which the oracle receives exactly)."""
    from capk import ops
    g = torch.Generator().manual_seed(V)
    R = 48
    x = (torch.randn(R, V, generator=g) * scale).to(dtype).float()
    ld = (V + 63) // 64 * 64
    xp = torch.full((R, ld), 1e4)
    xp[:, :V] = x
    xp = xp.to(dtype)
    out = torch.empty(R, dtype=torch.long, device="cuda")
    logp = torch.empty(R, dtype=torch.float32, device="cuda")
    for step in (0, 7):
        ops.sample_rows(xp.cuda(), V, 1234, step, out, logp)
        got, glp = out.cpu().numpy(), logp.cpu().numpy()
        for r in range(R):
            tok, lp, margin = oscst.sample_row(x[r].numpy(), 1234, step, r)
            if margin > 1e-5:
                assert got[r] == tok, (step, r, got[r], tok, margin)
                assert abs(glp[r] - lp) < 1e-4 * max(1.0, abs(lp))
    # empirical distribution: many draws of one row follow softmax
    row = (torch.randn(1, 64, generator=g) * 0.7).repeat(4096, 1)
    ops.sample_rows(row.cuda(), 64, 99, 0, out.new_empty(4096), None)
    draws = torch.empty(4096, dtype=torch.long, device="cuda")
    ops.sample_rows(row.cuda(), 64, 99, 3, draws, None)
    freq = torch.bincount(draws.cpu(), minlength=64).float() / 4096
    assert float((freq - torch.softmax(row[0], 0)).abs().max()) < 0.03


@cuda
def test_weighted_ce_kernel():
    from capk.train.scst import policy_gradient_loss, pg_targets
    g = torch.Generator().manual_seed(0)
    B, T, V = 5, 7, 100
    logits = torch.randn(B, T, V, generator=g)
    ids = torch.randint(0, V, (B, T), generator=g)
    ids[1, 3] = 99
    ids[3, 1] = 99
    adv = torch.randn(B, generator=g)
    ld = 128
    buf = torch.zeros(B * T, ld)
    buf[:, :V] = logits.view(B * T, V)
    lg = buf.cuda().requires_grad_(True)
    view = lg[:, :V].view(B, T, V)
    loss = policy_gradient_loss(view, ids.cuda(), adv.cuda(), 99)
    loss.backward()
    ref_l = logits.clone().requires_grad_(True)
    tgt = pg_targets(ids, 99)
    lp = F.log_softmax(ref_l[:, :-1], -1).gather(-1, tgt[:, 1:].clamp(min=0)[..., None])[..., 0]
    mask = (tgt[:, 1:] != -100).float()
    ref = -(lp * adv[:, None] * mask).sum() / mask.sum()
    ref.backward()
    torch.testing.assert_close(loss.detach().cpu(), ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(lg.grad.cpu()[:, :V].view(B, T, V), ref_l.grad, rtol=1e-4, atol=1e-6)
    assert float(mask[1, 3:].sum()) == 0.0 and float(mask[1, 2]) == 1.0  # tokens after the first EOS ignored


def _tiny():
    from test_gpu_model import _tiny_model
    z = np.load(os.path.join(GOLD, "vit_transformer_step.npz"), allow_pickle=False)
    model, store, cfg = _tiny_model(z, "fp32")
    return z, model, store, cfg


@cuda
def test_scst_sampling_and_update_vs_oracle():
    from capk.train import CapkAdamW
    from capk.train.scst import pg_targets, sample_captions, scst_step, strip_special, cider_d
    from oracle import decoders as odec
    from oracle import encoders as oenc
    z, model, store, cfg = _tiny()
    D, Le, He, Ld, Hd, V, pad, patch, img = [int(x) for x in z["meta/dims"]]
    images = torch.from_numpy(z["in/images"]).cuda()
    B = images.shape[0]
    sd = {k: v.detach().cpu().float().clone() for k, v in model.state_dict().items()}
    with torch.no_grad():
        enc = model.encoder(images)
        ids, logp = sample_captions(model.decoder, enc, 9, seed=77)
    # oracle sampler over the oracle decoder
    p = {k[len("decoder."):]: v for k, v in sd.items() if k.startswith("decoder.")}
    with torch.no_grad():
        feats = oenc.vit_encoder({k[len("encoder.model."):]: v for k, v in sd.items()
                                  if k.startswith("encoder.model.")}, images.cpu(), Le, He, patch)["features"]
        mem = F.linear(feats, p["visual_projection.weight"], p["visual_projection.bias"])
        oids = torch.full((B, 1), pad, dtype=torch.long)
        for t in range(8):
            lg = odec.transformer_last_logits(p, mem, oids, Ld, Hd)
            nxt = torch.tensor([oscst.sample_row(lg[r].numpy(), 77, t, r)[0] for r in range(B)])
            oids = torch.cat([oids, nxt[:, None]], 1)
            if bool((nxt == pad).all()):
                break
    assert torch.equal(ids.cpu(), oids)
    # one SCST update: loss + every gradient vs autograd of the oracle decoder (encoder frozen in the check)
    refs = [[[3, 5, 7, 9]], [[1, 2, 3]], [[4, 4, 8, 15, 16]]]
    opt = CapkAdamW(store, lr=0.0, weight_decay=0.0)
    loss, rs, rb = scst_step(model, images, refs, opt, lr=0.0, max_length=9, seed=77)
    samp = [strip_special(r, pad, pad, pad) for r in ids.cpu().tolist()]
    with torch.no_grad():
        base_ids, _ = model.decoder.generate({"features": enc["features"]}, 9)
    base = [strip_special(r, pad, pad, pad) for r in base_ids.cpu().tolist()]
    adv = torch.tensor(cider_d(samp, refs) - cider_d(base, refs), dtype=torch.float32)
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    memr = F.linear(feats, pr["visual_projection.weight"], pr["visual_projection.bias"])
    T1 = ids.shape[1]
    x = pr["embedding.weight"][ids.cpu()] + pr["position_encoding.weight"][:T1][None]
    for i in range(Ld):
        x = odec.decoder_layer(pr, i, x, memr, Hd, None)
    logits = F.linear(x, pr["output_layer.weight"], pr["output_layer.bias"])
    tgt = pg_targets(ids.cpu(), pad)
    lp = F.log_softmax(logits[:, :-1], -1).gather(-1, tgt[:, 1:].clamp(min=0)[..., None])[..., 0]
    mask = (tgt[:, 1:] != -100).float()
    ref = -(lp * adv[:, None] * mask).sum() / mask.sum()
    ref.backward()
    pr["embedding.weight"].grad[pad] = 0.0  # nn.Embedding(padding_idx=pad): no gradient for the pad row
    torch.testing.assert_close(loss.cpu(), ref.detach(), rtol=1e-4, atol=1e-6)
    for n, prm in model.decoder.named_parameters():
        if pr[n].grad is None:
            continue
        gref = pr[n].grad
        torch.testing.assert_close(prm._capk_grad.cpu(), gref, rtol=2e-3, atol=2e-3 * float(gref.abs().max()) + 1e-8,
                                   msg=lambda m: f"{n}: {m}")


@cuda
def test_scst_concurrent_baseline_equals_sequential():
    """The baseline search on a side stream / host thread, concurrent with the sampler
    (capk.train.scst.CONCURRENT, from a decoder's second update on), gives exactly the
    sequential update: same losses and rewards over three updates (eager first, then graph
    capture and replay of both decode loops while the other runs)."""
    from capk import graphs
    from capk.train import CapkAdamW
    from capk.train import scst as S
    refs = [[[3, 5, 7, 9]], [[1, 2, 3]], [[4, 4, 8, 15, 16]]]
    out = {}
    old = S.CONCURRENT
    try:
        for mode in (False, True):
            S.CONCURRENT = mode
            S._WARM.clear()
            graphs.clear()
            z, model, store, cfg = _tiny()
            images = torch.from_numpy(z["in/images"]).cuda()
            opt = CapkAdamW(store, lr=1e-3, weight_decay=0.0)
            res = []
            for it in range(3):
                loss, rs, rb = S.scst_step(model, images, refs, opt, lr=1e-3, max_length=9, seed=100 + it)
                res.append((float(loss), rs, rb))
            out[mode] = res
    finally:
        S.CONCURRENT = old
        S._WARM.clear()
        graphs.clear()
    assert out[True] == out[False], out
