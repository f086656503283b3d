"""Swin encoder (src/models/encoders.py:140-182) on the GPU.

* window attention kernels vs a plain torch fp32 reference of the same op (shifted and
  unshifted windows, relative-position bias, fp32 <= 1e-5 / bf16 <= 2e-2 relative),
  including the relative-position-table gradient;
* fp32 SwinEncoder vs tests/golden/swin_encoder.npz (the reference's own SwinEncoder over a
  random-init transformers SwinModel, oracle/gen_golden.py): features / pooled (rtol 1e-4)
  and every parameter gradient (rtol 2e-4 of the tensor's max);
* SwinDropPath with a fixed per-sample factor vs the oracle with the same factor;
* full-size Swin-B (microsoft/swin-base-patch4-window7-224 architecture) in bf16 vs the fp32
  oracle on the same weights: features <= 3e-2 relative;
* ImageCaptioningModel with encoder_type="swin": bf16 train step (finite, gradients reach
  the patch embedding) and greedy generate.
"""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "swin_encoder.npz")


def _rel(a, b):
    a, b = a.detach().float().cpu(), torch.as_tensor(b).float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _ref_window_attn(qkv, C, H, ws, labels, table):
    """torch fp32 reference: window-ordered rows, scores + rel bias (+ -100 shift mask)."""
    from oracle.encoders import _swin_rel_index
    N = ws * ws
    hd = C // H
    x = qkv.float().view(-1, N, 3, H, hd)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))  # [nwin, H, N, hd]
    s = q @ k.transpose(-1, -2) * hd ** -0.5
    s = s + table.float()[_swin_rel_index(ws).reshape(-1).to(table.device)].view(N, N, H).permute(2, 0, 1)
    if labels is not None:
        nW = labels.shape[0]
        m = (labels[:, :, None] != labels[:, None, :]).float() * -100.0
        s = (s.view(-1, nW, H, N, N) + m[None, :, None]).view(-1, H, N, N)
    o = torch.softmax(s, -1) @ v
    return o.transpose(1, 2).reshape(-1, C)


@cuda
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shift", [0, 3])
def test_window_attention_fwd_bwd_vs_torch(dtype, shift):
    from capk import ops
    from capk.models.swin import shift_labels
    torch.manual_seed(0)
    B, Hs, ws, H = 3, 14, 7, 4
    C = 32 * H
    N = ws * ws
    rows = B * Hs * Hs
    qkv = torch.randn(rows, 3 * C, device="cuda").to(dtype)
    table = (torch.randn((2 * ws - 1) ** 2, H, device="cuda") * 0.5)
    labels = None
    if shift:
        labels = torch.from_numpy(np.ascontiguousarray(shift_labels(Hs, Hs, ws, shift), dtype=np.int32)).cuda()
    out = torch.empty(rows, C, device="cuda", dtype=dtype)
    lse = ops.window_attn_fwd(qkv, C, H, ws, (Hs // ws) ** 2, 32 ** -0.5, table, labels, out)
    q32 = qkv.float().requires_grad_(True)
    t32 = table.clone().requires_grad_(True)
    ref = _ref_window_attn(q32, C, H, ws, labels, t32)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(out, ref) < tol, _rel(out, ref)
    dout = torch.randn(rows, C, device="cuda").to(dtype)
    ref.backward(dout.float())
    dqkv = torch.empty_like(qkv)
    dtab = torch.zeros_like(table)
    ops.window_attn_bwd(qkv, C, H, ws, (Hs // ws) ** 2, 32 ** -0.5, table, labels, out, dout, lse, dqkv, dtab)
    torch.cuda.synchronize()
    for i, name in enumerate("qkv"):
        got = dqkv[:, i * C:(i + 1) * C]
        want = q32.grad[:, i * C:(i + 1) * C]
        assert _rel(got, want) < (2e-5 if dtype == torch.float32 else 3e-2), (name, _rel(got, want))
    assert _rel(dtab, t32.grad) < (2e-5 if dtype == torch.float32 else 3e-2), _rel(dtab, t32.grad)
    assert lse.shape == (B * (Hs // ws) ** 2, H, N)


def _arch_from_fixture(z):
    img, P, E, ws, Fd, B = [int(x) for x in z["meta/dims"]]
    return dict(image_size=img, patch_size=P, num_channels=3, embed_dim=E, depths=tuple(int(x) for x in z["meta/depths"]),
                num_heads=tuple(int(x) for x in z["meta/heads"]), window_size=ws, mlp_ratio=4.0, qkv_bias=True,
                layer_norm_eps=1e-5, drop_path_rate=0.1), Fd


def _golden_encoder(z, precision):
    import capk
    from capk import config as C
    from capk.models.encoders import SwinEncoder
    arch, Fd = _arch_from_fixture(z)
    enc = SwinEncoder(C.EncoderConfig(encoder_type="swin", feature_dim=Fd), arch=arch)
    sd = {k[3:]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("p0/")}
    enc.load_state_dict(sd, strict=True)
    capk.prepare(enc, "cuda", precision)
    return enc, sd


@cuda
def test_swin_encoder_golden_fp32():
    z = np.load(GOLD, allow_pickle=False)
    enc, _ = _golden_encoder(z, "fp32")
    enc.eval()
    out = enc(torch.from_numpy(z["in/images"]).cuda())
    np.testing.assert_allclose(out["features"].detach().cpu().numpy(), z["out/features"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(out["pooled_features"].detach().cpu().numpy(), z["out/pooled"], rtol=1e-4, atol=1e-5)
    assert out["attention_mask"].all() and out["attention_mask"].shape == z["out/mask"].shape
    loss = (out["features"] * torch.from_numpy(z["in/gf"]).cuda()).sum() + \
        (out["pooled_features"] * torch.from_numpy(z["in/gp"]).cuda()).sum()
    loss.backward()
    torch.cuda.synchronize()
    for n, p in enc.named_parameters():
        ref = z["grad/" + n]
        got = p._capk_grad.detach().cpu().numpy().reshape(ref.shape)
        np.testing.assert_allclose(got, ref, rtol=2e-4, atol=2e-4 * float(np.abs(ref).max()) + 1e-7, err_msg=n)


@cuda
def test_swin_drop_path_matches_oracle_with_same_keep():
    """SwinDropPath on the attention branch (modeling_swin.py:42-60, 567) with the per-sample
    factor fixed on both sides (the factor's RNG is torch's and is not compared)."""
    from capk.models import swin as S
    from oracle import encoders as oenc
    z = np.load(GOLD, allow_pickle=False)
    enc, sd = _golden_encoder(z, "fp32")
    enc.train()
    B = z["in/images"].shape[0]
    nblk = sum(int(x) for x in z["meta/depths"])
    g = torch.Generator().manual_seed(5)
    keeps = [(torch.rand(B, generator=g) < 0.6).float() / 0.6 for _ in range(nblk)]
    it = iter(keeps)
    orig = S._drop_path_scale
    S._drop_path_scale = lambda L, Bn, dev: next(it).to(dev)
    try:
        out = enc(torch.from_numpy(z["in/images"]).cuda())
    finally:
        S._drop_path_scale = orig
    depths = [int(x) for x in z["meta/depths"]]
    heads = [int(x) for x in z["meta/heads"]]
    p = {k: v.requires_grad_(True) for k, v in sd.items()}
    f, pooled = oenc.swin_encoder(p, torch.from_numpy(z["in/images"]), depths, heads, keep=keeps)
    assert _rel(out["features"], f) < 1e-5, _rel(out["features"], f)
    gf = torch.from_numpy(z["in/gf"])
    (out["features"] * gf.cuda()).sum().backward()
    (f * gf).sum().backward()
    torch.cuda.synchronize()
    for n, prm in enc.named_parameters():
        if p[n].grad is None or float(p[n].grad.abs().max()) < 1e-6:
            continue
        assert _rel(prm._capk_grad.view(p[n].shape), p[n].grad) < 1e-4, n


@cuda
def test_swin_base_bf16_vs_oracle():
    """The reference default architecture (encoders.py:146-147) at 224x224, bf16 vs fp32 oracle."""
    import capk
    from capk import config as C
    from capk.models.encoders import SwinEncoder
    from oracle import encoders as oenc
    torch.manual_seed(11)
    enc = SwinEncoder(C.EncoderConfig(encoder_type="swin", feature_dim=768,
                                      pretrained_model_name="microsoft/swin-base-patch4-window7-224"))
    with torch.no_grad():
        for n, p in enc.named_parameters():
            if n.endswith("relative_position_bias_table"):
                p.normal_(0.0, 0.5)
    sd = {k: v.detach().clone() for k, v in enc.state_dict().items()}
    capk.prepare(enc, "cuda", "bf16")
    enc.eval()
    B = 2
    images = torch.randn(B, 3, 224, 224)
    out = enc(images.cuda())
    assert out["features"].shape == (B, 49, 768) and out["pooled_features"].shape == (B, 768)
    f, pooled = oenc.swin_encoder(sd, images, [2, 2, 18, 2], [4, 8, 16, 32])
    assert _rel(out["features"], f) < 3e-2, _rel(out["features"], f)
    assert _rel(out["pooled_features"], pooled) < 3e-2, _rel(out["pooled_features"], pooled)


@cuda
def test_captioning_model_with_swin_trains_and_generates():
    import capk
    from capk import config as C
    from capk.models import captioning_model as cm
    from capk.train import CapkAdamW, CombinedLoss
    torch.manual_seed(4)
    cfg = C.Config()
    cfg.model.encoder = C.EncoderConfig(encoder_type="swin", pretrained_model_name="microsoft/swin-tiny-patch4-window7-224")
    cfg.model.decoder = C.DecoderConfig(decoder_type="transformer", hidden_dim=768, num_layers=2, num_heads=8)
    cfg.model.vocab_size, cfg.model.pad_token_id = 50257, 50256
    cfg.model.bos_token_id = cfg.model.eos_token_id = 50256
    model = cm.ImageCaptioningModel(cfg)
    store = capk.prepare(model, "cuda", "bf16")
    model.train()
    B, T = 4, 12
    images = torch.randn(B, 3, 224, 224, device="cuda")
    caps = torch.randint(0, 50256, (B, T), device="cuda")
    opt = CapkAdamW(store, lr=1e-4)
    losses = []
    for _ in range(2):
        out = model(images=images, captions=caps)
        loss = CombinedLoss(50256)(out["logits"], caps)["total_loss"]
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert all(math.isfinite(x) for x in losses)
    g = model.encoder.model.embeddings.patch_embeddings.projection.weight._capk_grad
    assert torch.isfinite(g).all() and float(g.abs().max()) > 0
    model.eval()
    ids, _ = model.generate(images=images, max_length=5)
    assert ids.shape[0] == B


@cuda
@pytest.mark.parametrize("M", [6272, 300])
def test_bf16_gemm_k96_vs_torch(M):
    """Swin-T/S widths (C = 96): K-major bf16 products with K % 64 != 0 run on the BK-32 rings."""
    from capk import ops
    torch.manual_seed(2)
    K, N = 96, 288
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
    b = torch.randn(N, device="cuda")
    y = ops.linear(x, w, b)
    ref = x.float() @ w.float().t() + b
    assert _rel(y, ref) < 1e-2, _rel(y, ref)
    dy = torch.randn(M, N, device="cuda").bfloat16()
    dx = ops.linear_dx(dy, w)  # contraction over N = 288 (% 64 != 0) with a K-major dY
    assert _rel(dx, dy.float() @ w.float()) < 1e-2
