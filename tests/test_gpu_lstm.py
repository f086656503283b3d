"""LSTM decoder (A6) with the attention modules (A7-A10) on the GPU vs the reference's
own outputs (tests/golden/lstm_attention.npz, oracle/gen_golden.py): logits, attention
weights, loss, every parameter gradient, d(features), d(pooled) and greedy ids (fp32);
bf16 logits within 3e-2; bf16 train-mode steps reduce the loss."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lstm_attention.npz")
VARIANTS = {"soft": ("soft", 1, 0.7), "multi_head": ("multi_head", 4, 1.0), "aoa": ("aoa", 4, 1.0),
            "adaptive": ("adaptive", 4, 1.0), "adaptive_soft": ("adaptive", 1, 1.0)}


def _decoder(name, precision):
    import capk
    from capk import config as C
    from capk.models.decoders import build_decoder
    z = np.load(GOLD, allow_pickle=False)
    D, L, V, B, T, S, pad = [int(x) for x in z["meta/dims"]]
    kind, heads, temp = VARIANTS[name]
    dec = build_decoder(C.DecoderConfig(decoder_type="lstm", hidden_dim=D, num_layers=L, num_heads=heads, dropout=0.1),
                        C.AttentionConfig(attention_type=kind, num_heads=heads, temperature=temp), V, pad, pad, pad)
    pre = name + "/p0/"
    sd = {k[len(pre):]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith(pre)}
    dec.load_state_dict(sd, strict=True)
    capk.prepare(dec, "cuda", precision)
    dec.eval()
    return z, dec


@cuda
@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_lstm_golden_fp32(name):
    from capk.train import CombinedLoss
    z, dec = _decoder(name, "fp32")
    D, L, V, B, T, S, pad = [int(x) for x in z["meta/dims"]]
    feats = torch.from_numpy(z["in/features"]).cuda().requires_grad_(True)
    pooled = torch.from_numpy(z["in/pooled"]).cuda().requires_grad_(True)
    caps = torch.from_numpy(z["in/captions"]).cuda()
    out = dec({"features": feats, "pooled_features": pooled, "attention_mask": None}, caps)
    np.testing.assert_allclose(out["logits"].detach().cpu().numpy(), z[name + "/logits"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["attention_weights"].detach().cpu().numpy(), z[name + "/attention_weights"],
                               rtol=1e-4, atol=1e-6)
    loss = CombinedLoss(pad)(logits=out["logits"], targets=caps)["total_loss"]
    np.testing.assert_allclose(float(loss), float(z[name + "/loss"][0]), rtol=1e-5)
    loss.backward()
    for ref_key, got in ((name + "/dfeatures", feats.grad), (name + "/dpooled", pooled.grad)):
        ref = z[ref_key]
        np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=2e-4, atol=2e-4 * float(np.abs(ref).max()),
                                   err_msg=ref_key)
    for n, p in dec.named_parameters():
        key = name + "/grad/" + n
        ref = z[key]
        np.testing.assert_allclose(p._capk_grad.cpu().numpy(), ref, rtol=2e-4,
                                   atol=2e-4 * float(np.abs(ref).max()) + 1e-8, err_msg=n)
    with torch.no_grad():
        ids, info = dec.generate({"features": feats.detach(), "pooled_features": pooled.detach()}, 6,
                                 start_token_id=pad)
    np.testing.assert_array_equal(ids.cpu().numpy(), z[name + "/greedy_ids"])


@cuda
def test_standalone_attention_modules_fp32():
    """AttentionMechanism.forward(query, key, value) drop-in contract (attention.py:12-35)
    for soft / multi_head / aoa against the oracle restatement, with gradients."""
    import torch.nn.functional as F  # noqa: F401
    import capk
    from capk import config as C
    from capk.models.attention import build_attention
    from oracle import lstm as olstm
    torch.manual_seed(3)
    B, S, D = 3, 9, 64
    for kind, heads in (("soft", 1), ("multi_head", 4), ("aoa", 4)):
        cfg = C.AttentionConfig(attention_type=kind, num_heads=heads, temperature=1.3)
        cfg.hidden_dim = D
        mod = build_attention(cfg)
        sd = {k: v.detach().clone() for k, v in mod.state_dict().items()}
        capk.prepare(mod, "cuda", "fp32")
        q = torch.randn(B, D).cuda().requires_grad_(True)
        kv = torch.randn(B, S, D).cuda().requires_grad_(True)
        ctx, w = mod(q, kv, kv)
        wl = 1.0 if kind == "soft" else 0.0  # MHA/AoA weights are returned for inspection (no gradient)
        (ctx.square().sum() + wl * (w * torch.arange(S, device="cuda")).sum()).backward()
        p = {"attention." + k: v.clone().requires_grad_(True) for k, v in sd.items()}
        qr = q.detach().cpu().requires_grad_(True)
        kr = kv.detach().cpu().requires_grad_(True)
        rc, rw = olstm.attend(kind, p, qr, kr, heads, 1.3, None, None)
        (rc.square().sum() + wl * (rw * torch.arange(S)).sum()).backward()
        torch.testing.assert_close(ctx.detach().cpu(), rc.detach(), rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(w.detach().cpu(), rw.detach(), rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(q.grad.cpu(), qr.grad, rtol=1e-3, atol=1e-5)
        torch.testing.assert_close(kv.grad.cpu(), kr.grad, rtol=1e-3, atol=1e-5)
        for n, prm in mod.named_parameters():
            torch.testing.assert_close(prm._capk_grad.cpu(), p["attention." + n].grad, rtol=1e-3, atol=1e-5,
                                       msg=lambda m: f"{kind} {n}: {m}")


@cuda
@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_lstm_bf16_close_and_trains(name):
    from capk.train import CapkAdamW, CombinedLoss
    z, dec = _decoder(name, "bf16")
    D, L, V, B, T, S, pad = [int(x) for x in z["meta/dims"]]
    feats = torch.from_numpy(z["in/features"]).cuda().bfloat16()
    pooled = torch.from_numpy(z["in/pooled"]).cuda().bfloat16()
    caps = torch.from_numpy(z["in/captions"]).cuda()
    enc = {"features": feats, "pooled_features": pooled, "attention_mask": None}
    with torch.no_grad():
        got = dec(enc, caps)["logits"].float().cpu()
    ref = torch.from_numpy(z[name + "/logits"])
    assert float((got - ref).norm() / ref.norm()) < 3e-2
    dec.train()
    store = next(iter(dec.parameters()))._capk_store_ref
    opt = CapkAdamW(store, lr=3e-3, weight_decay=0.01)
    lf = CombinedLoss(pad)
    losses = []
    for _ in range(8):
        loss = lf(logits=dec(enc, caps)["logits"], targets=caps)["total_loss"]
        loss.backward()
        opt.step(lr=3e-3)
        losses.append(float(loss))
    assert all(np.isfinite(losses)) and losses[-1] < losses[0] * 0.9, losses


def _full_lstm(precision, kind="soft", heads=1, seed=21, embedding_dim=None):
    """Config-2 decoder geometry: LSTM 768 hidden x 6 layers (DecoderConfig defaults),
    soft attention over the 49 ResNet feature keys, GPT-2 vocabulary (embedding_dim: the
    reference LSTMDecoder's optional embedding width, decoders.py:77-100)."""
    import capk
    from capk import config as C
    from capk.models.decoders import build_decoder
    from capk.models.decoders import LSTMDecoder
    torch.manual_seed(seed)
    V, pad = 50257, 50256
    dcfg = C.DecoderConfig(decoder_type="lstm", hidden_dim=768, num_layers=6, num_heads=heads)
    acfg = C.AttentionConfig(attention_type=kind, num_heads=heads)
    acfg.hidden_dim = 768
    if embedding_dim is None:
        dec = build_decoder(dcfg, acfg, V, pad, pad, pad)
    else:
        dec = LSTMDecoder(dcfg, acfg, V, pad, embedding_dim=embedding_dim)
    sd = {k: v.detach().clone() for k, v in dec.state_dict().items()}
    capk.prepare(dec, "cuda", precision)
    dec.eval()
    return dec, sd


@cuda
@pytest.mark.parametrize("precision,tol", [("fp32", 1e-3), ("bf16", 3e-2)])
def test_lstm_full_size_vs_oracle(precision, tol):
    """768 hidden, 6 layers, 49 keys, batch 8, 20 tokens vs oracle/lstm.py (fp32 CPU):
    logits and attention weights within the north-star 1e-3 (fp32) / 3e-2 (bf16) relative;
    fp32 gradients of features, pooled and the LSTM / attention weights within 1e-3."""
    from oracle import lstm as olstm
    from capk.train import CombinedLoss
    dec, sd = _full_lstm(precision)
    B, T, S, D = 8, 20, 49, 768
    g = torch.Generator().manual_seed(2)
    feats = torch.randn(B, S, D, generator=g)
    pooled = torch.randn(B, D, generator=g)
    caps = torch.randint(0, 50256, (B, T), generator=g)
    dt = torch.float32 if precision == "fp32" else torch.bfloat16
    fg = feats.cuda().to(dt).requires_grad_(True)
    pg = pooled.cuda().to(dt).requires_grad_(True)
    out = dec({"features": fg, "pooled_features": pg, "attention_mask": None}, caps.cuda())
    p = {k: v.float().requires_grad_(True) for k, v in sd.items()}
    fr = fg.detach().float().cpu().requires_grad_(True)
    pr = pg.detach().float().cpu().requires_grad_(True)
    ref_logits, ref_w = olstm.lstm_decoder(p, fr, pr, caps, 6, "soft")

    def rel(a, b):
        return float((a.detach().float().cpu() - b.detach()).norm() / b.detach().norm())

    assert rel(out["logits"], ref_logits) < tol
    assert rel(out["attention_weights"], ref_w) < tol
    if precision == "fp32":
        loss = CombinedLoss(50256)(logits=out["logits"], targets=caps.cuda())["total_loss"]
        loss.backward()
        from oracle.train import shifted_ce
        ref_loss = shifted_ce(ref_logits, caps, 50256)
        ref_loss.backward()
        assert abs(float(loss) - float(ref_loss)) < 1e-4 * abs(float(ref_loss))
        assert rel(fg.grad, fr.grad) < 1e-3 and rel(pg.grad, pr.grad) < 1e-3
        for n, prm in dec.named_parameters():
            if p[n].grad is not None:  # (the attention energy bias shifts every key equally: its
                # true gradient is 0 and both sides hold rounding noise -> absolute floor)
                ref = p[n].grad
                err = float((prm._capk_grad.float().cpu() - ref).norm())
                assert err <= 1e-3 * float(ref.norm()) + 1e-6, (n, err, float(ref.norm()))


@cuda
def test_gemm_pair_slabs_k_and_n_seams():
    """capk_gemm_pair_slabs: the slabs sum to [A | A2] [B | B2]^T (K seam, both K-major) and
    to [A B^T | A B2^T] (N seam, N-major B as in dX = dG W) -- fp32 accumulation of bf16
    products, compared with the fp32 product of the same bf16 values."""
    from capk import ops
    torch.manual_seed(5)
    M, D = 128, 768
    bf = torch.bfloat16
    x, h = torch.randn(M, D, device="cuda", dtype=bf), torch.randn(M, D, device="cuda", dtype=bf)
    wi, wh = torch.randn(4 * D, D, device="cuda", dtype=bf), torch.randn(4 * D, D, device="cuda", dtype=bf)
    s, n = ops.pair_slabs_plan(M, 4 * D, 2 * D)
    ws = torch.full((n,), float("nan"), device="cuda")
    got_s = ops.gemm_pair_slabs(M, 4 * D, 2 * D, x, D, wi, D, True, ws, A2=h, lda2=D, B2=wh, ldb2=D, k1=D)
    assert got_s == s and s > 1
    got = ws[:s * M * 4 * D].view(s, M, 4 * D).sum(0)
    ref = x.float() @ wi.float().t() + h.float() @ wh.float().t()
    assert float((got - ref).norm() / ref.norm()) < 1e-5
    # N seam: dG [M, 4D] against W_ih, W_hh as N-major operands -> [dG W_ih | dG W_hh]
    dg = torch.randn(M, 4 * D, device="cuda", dtype=bf)
    s, n = ops.pair_slabs_plan(M, 2 * D, 4 * D)
    ws = torch.full((n,), float("nan"), device="cuda")
    assert ops.gemm_pair_slabs(M, 2 * D, 4 * D, dg, 4 * D, wi, D, False, ws, B2=wh, ldb2=D, n1=D) == s
    got = ws[:s * M * 2 * D].view(s, M, 2 * D).sum(0)
    ref = torch.cat([dg.float() @ wi.float(), dg.float() @ wh.float()], 1)
    assert float((got - ref).norm() / ref.norm()) < 1e-5
    out = torch.empty(M, D, device="cuda", dtype=bf)
    ops.slab_sum(ws, s, M, 2 * D, D, out)
    assert float((out.float() - ref[:, D:]).norm() / ref[:, D:].norm()) < 4e-3
    res = torch.randn(M, D, device="cuda", dtype=bf)
    ops.slab_sum(ws, s, M, 2 * D, 0, out, res=res)
    want = ref[:, :D] + res.float()
    assert float((out.float() - want).norm() / want.norm()) < 4e-3


@cuda
@pytest.mark.parametrize("embedding_dim", [None, 320])
def test_lstm_pair_route_matches_gemm_route_train_bf16(embedding_dim):
    """The bf16 teacher-forced pass with the pair-slab recurrences (default) against the
    per-GEMM route (two GEMMs + reduces per step and layer) on the same weights, inputs and
    dropout seeds, in train mode at the config-2 geometry (768 x 6 layers, inter-layer and
    output dropout on): logits, d(features), d(pooled) and every parameter gradient within
    3e-2 relative (bf16 rounding of the two routes differs: fp32 slab sums vs bf16 gates).
    embedding_dim 320 ((E + D) % 128 != 0) takes the mixed backward: layer 0 on the per-GEMM
    route (dnext by its own product, dh[0] carried as the initial-state gradient) under the
    slab-summed upper layers."""
    import capk.models.lstm as mlstm
    from capk.models import common
    from capk.train import CombinedLoss
    dec, _ = _full_lstm("bf16", embedding_dim=embedding_dim)
    dec.train()
    B, T, S, D = 16, 20, 49, 768
    g = torch.Generator().manual_seed(4)
    feats = torch.randn(B, S, D, generator=g).cuda().bfloat16()
    pooled = torch.randn(B, D, generator=g).cuda().bfloat16()
    caps = torch.randint(0, 50256, (B, T), generator=g).cuda()
    runs = []
    saved = mlstm._PAIR
    try:
        for pair in (True, False):
            mlstm._PAIR = pair
            common._SEED[0] = 777
            for p in dec.parameters():
                if getattr(p, "_capk_grad", None) is not None:
                    p._capk_grad.zero_()
            fg = feats.clone().requires_grad_(True)
            pg = pooled.clone().requires_grad_(True)
            out = dec({"features": fg, "pooled_features": pg, "attention_mask": None}, caps)
            loss = CombinedLoss(50256)(logits=out["logits"], targets=caps)["total_loss"]
            loss.backward()
            grads = {n: p._capk_grad.float().clone() for n, p in dec.named_parameters()
                     if getattr(p, "_capk_grad", None) is not None}
            runs.append((out["logits"].detach().float(), fg.grad.float(), pg.grad.float(), grads))
    finally:
        mlstm._PAIR = saved

    def rel(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    (la, fa, pa, ga), (lb, fb, pb, gb) = runs
    assert rel(la, lb) < 3e-2 and rel(fa, fb) < 3e-2 and rel(pa, pb) < 3e-2
    checked = 0
    for n, ref in gb.items():
        if float(ref.norm()) == 0.0:
            continue
        if n.startswith("lstm.") or n.startswith("init_") or n.startswith("attention."):
            err = float((ga[n] - ref).norm())
            # the attention energy bias has a true gradient of 0: absolute floor
            assert err <= 3e-2 * float(ref.norm()) + 1e-3, (n, err, float(ref.norm()))
            checked += 1
    assert checked >= 4 * 6


@cuda
@pytest.mark.parametrize("precision,tol", [("fp32", 1e-6), ("bf16", 1e-3)])
def test_soft_attention_deferred_kv_grad_matches_per_step(precision, tol):
    """The soft-attention backward's deferred key / value gradients (default: each decode step
    stashes d(energy) [B, S] and d(context) [B, D]; capk_soft_attn_kv_grad writes dK / dV once
    after the last step, summing in the per-step order) against the per-step read-modify-write
    route (CAPK_SOFT_DEFER=0) on the same weights and inputs at the config-2 geometry (768 x 6,
    49 keys): d(features), d(pooled) and every attention / LSTM gradient agree to `tol`
    (relative; bit-identity is reported, the claim of attention.py's deferral)."""
    import capk.models.attention as matt
    from capk.train import CombinedLoss
    dec, _ = _full_lstm(precision)
    B, T, S, D = 8, 20, 49, 768
    g = torch.Generator().manual_seed(6)
    dt = torch.float32 if precision == "fp32" else torch.bfloat16
    feats = torch.randn(B, S, D, generator=g).cuda().to(dt)
    pooled = torch.randn(B, D, generator=g).cuda().to(dt)
    caps = torch.randint(0, 50256, (B, T), generator=g).cuda()
    runs = []
    saved = matt._SOFT_DEFER
    try:
        for defer in (True, False):
            matt._SOFT_DEFER = defer
            for p in dec.parameters():
                if getattr(p, "_capk_grad", None) is not None:
                    p._capk_grad.zero_()
            fg = feats.clone().requires_grad_(True)
            pg = pooled.clone().requires_grad_(True)
            out = dec({"features": fg, "pooled_features": pg, "attention_mask": None}, caps)
            CombinedLoss(50256)(logits=out["logits"], targets=caps)["total_loss"].backward()
            grads = {n: p._capk_grad.float().clone() for n, p in dec.named_parameters()
                     if getattr(p, "_capk_grad", None) is not None}
            runs.append((fg.grad.float(), pg.grad.float(), grads))
    finally:
        matt._SOFT_DEFER = saved
    (fa, pa, ga), (fb, pb, gb) = runs
    same = torch.equal(fa, fb) and torch.equal(pa, pb) and all(torch.equal(ga[n], gb[n]) for n in gb)
    print(f"soft deferral {precision}: bit-identical={same}")

    def rel(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    assert rel(fa, fb) <= tol and rel(pa, pb) <= tol
    checked = 0
    for n, ref in gb.items():
        if float(ref.norm()) == 0.0:
            continue
        assert float((ga[n] - ref).norm()) <= tol * float(ref.norm()) + 1e-7, n
        checked += 1
    assert checked >= 10
