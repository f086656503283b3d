"""The shifted cross entropy folded into the LM head (capk_linear_lse + capk_ce_lse_fwd /
capk_ce_lse_bwd; reference: src/train/losses.py:236-247 over src/models/decoders.py:431's
output_layer) against the separate route (capk_gemm + capk_shifted_ce + capk_colsum) and a
torch fp32 restatement of the loss on the same bf16 logits."""
import pytest
import torch

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")


def _case(seed=0, B=256, T=20, D=768, V=50257, Vp=50304):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(B * T, D, device="cuda", generator=g).bfloat16()
    w = torch.zeros(Vp, D, device="cuda")
    w[:V] = torch.randn(V, D, device="cuda", generator=g) * 0.05
    b = torch.zeros(Vp, device="cuda")
    b[:V] = torch.randn(V, device="cuda", generator=g) * 0.1
    tg = torch.randint(0, V - 1, (B, T), device="cuda", generator=g)
    tg[:, 15:] = V - 1  # padding tail (ignore_index = pad = V - 1)
    tg[::7, 9:] = V - 1
    return x, w.bfloat16().contiguous(), b, tg, V, Vp


@cuda
def test_lm_head_lse_loss_and_gradient():
    """Config-3 LM-head shape (5120 x 50 304 x 768, V = 50 257): the fused product's logits are
    bit-identical to capk_gemm's; the loss equals capk_shifted_ce's within 1e-5 and a torch
    fp32 log-softmax of the same bf16 logits within 1e-5; the row lse within 1e-4 of torch's;
    the gradient matches capk_shifted_ce's within bf16 rounding; the fused LM-head bias
    gradient equals the column sums of the gradient it wrote (fp32, 1e-5) and of the separate
    route's (1e-3 relative)."""
    from capk import ops
    x, w, b, tg, V, Vp = _case()
    B, T = tg.shape
    out, part = ops.linear_lse(x, w, b, V)
    assert part is not None, "the LM head shape must take the persistent kernel with partials"
    ref = ops.linear(x, w, b)
    assert torch.equal(out, ref)
    loss, lse = ops.ce_lse_fwd(out, tg, B, T, V, V - 1, part)
    loss_ref = ops.shifted_ce(ref, tg, B, T, V, V - 1, want_loss=True)
    assert float(loss[1]) == float(loss_ref[1])
    assert abs(float(loss[0]) - float(loss_ref[0])) <= 1e-5 * abs(float(loss_ref[0]))
    lg = out[:, :V].float()
    lse_t = torch.logsumexp(lg, -1)
    torch.testing.assert_close(lse, lse_t, rtol=1e-5, atol=1e-4)
    tgt = torch.cat([tg[:, 1:], torch.full((B, 1), V - 1, device="cuda")], 1).reshape(-1)
    keep = tgt != V - 1
    loss_t = (lse_t - lg.gather(1, tgt.clamp_max(V - 1)[:, None])[:, 0])[keep].mean()
    assert abs(float(loss[0]) - float(loss_t)) <= 1e-5 * abs(float(loss_t))
    gs = torch.full((1,), 0.5, device="cuda")
    d = torch.empty_like(out)
    db = torch.full((Vp,), 7.0, device="cuda")  # written, not accumulated
    ops.ce_lse_bwd(out, tg, B, T, V, V - 1, lse, loss, gs, d, db)
    d_ref = torch.empty_like(ref)
    ops.shifted_ce(ref, tg, B, T, V, V - 1, want_loss=False, dlogits=d_ref, grad_scale=gs)
    assert float((d.float() - d_ref.float()).abs().max()) <= 1e-3 * float(d_ref.float().abs().max())
    assert float(d[:, V:].abs().max()) == 0.0 and float(d[~keep].abs().max()) == 0.0
    torch.testing.assert_close(db, d.float().sum(0), rtol=1e-5, atol=1e-6)
    db_ref = torch.zeros(Vp, device="cuda")
    ops.colsum(d_ref, db_ref)
    assert float((db - db_ref).norm()) <= 1e-3 * float(db_ref.norm())


@cuda
def test_transformer_step_uses_fused_ce_and_matches_separate_route(monkeypatch):
    """A bf16 config-3-width Transformer decoder step (6 layers, V = 50 257, 64 images x 20
    tokens) through CombinedLoss: the fused route runs (partials merged, bias gradient written by
    the CE pass) and its loss, logits and every decoder gradient agree with the separate route
    (linear_lse disabled) within 1e-3 / 2e-2."""
    import capk
    from capk import config as C
    from capk import ops
    from capk.models.decoders import build_decoder
    from capk.train import CombinedLoss
    torch.manual_seed(3)
    V, pad = 50257, 50256
    dec = build_decoder(C.DecoderConfig(decoder_type="transformer"), C.AttentionConfig(), V, pad, pad, pad)
    capk.prepare(dec, "cuda", "bf16")
    dec.eval()  # no dropout: the two routes see the same masks
    B, T, S = 64, 20, 196
    g = torch.Generator().manual_seed(5)
    feats = torch.randn(B, S, 768, generator=g).cuda().bfloat16()
    caps = torch.randint(0, pad, (B, T), generator=g).cuda()
    caps[:, 16:] = pad
    calls = {"fwd": 0, "bwd": 0}
    f0, b0 = ops.ce_lse_fwd, ops.ce_lse_bwd

    def cf(*a, **k):
        calls["fwd"] += 1
        return f0(*a, **k)

    def cb(*a, **k):
        calls["bwd"] += 1
        return b0(*a, **k)

    monkeypatch.setattr(ops, "ce_lse_fwd", cf)
    monkeypatch.setattr(ops, "ce_lse_bwd", cb)
    runs = []
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(ops, "linear_lse", lambda x, w, b, V: (ops.linear(x, w, b), None))
        for p in dec.parameters():
            p._capk_grad.zero_()
        out = dec({"features": feats, "pooled_features": None, "attention_mask": None}, caps)
        loss = CombinedLoss(pad)(logits=out["logits"], targets=caps)["total_loss"]
        loss.backward()
        torch.cuda.synchronize()
        runs.append((float(loss), out["logits"].detach().float(),
                     {n: p._capk_grad.float().clone() for n, p in dec.named_parameters()}))
        if fused:
            assert calls == {"fwd": 1, "bwd": 1}, calls
    (la, ga_l, ga), (lb, gb_l, gb) = runs
    assert calls == {"fwd": 1, "bwd": 1}
    assert abs(la - lb) <= 1e-3 * abs(lb)
    torch.testing.assert_close(ga_l, gb_l, rtol=0, atol=0)
    for n, ref in gb.items():
        if float(ref.norm()) == 0.0:
            continue
        assert float((ga[n] - ref).norm()) <= 2e-2 * float(ref.norm()), n
