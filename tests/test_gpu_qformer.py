"""QFormer (src/models/captioning_model.py:153-245) on the GPU.

* fp32 vs tests/golden/qformer_step.npz (the reference's own QFormer, oracle/gen_golden.py):
  queries (rtol 1e-4), the feature gradient and every parameter gradient (rtol 2e-4);
* full size (768 wide, 32 queries, 8 heads, ViT-B/16 features with the CLS-row gap) in
  bf16 vs the fp32 oracle (oracle/encoders.py qformer): <= 3e-2 relative;
* ImageCaptioningModel with use_q_former=True (captioning_model.py:79-91): train step in
  bf16 with dropout, finite gradients reaching the encoder, and generate().
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "qformer_step.npz")


def _rel(a, b):
    a, b = a.detach().float().cpu(), torch.as_tensor(b).float()
    return float((a - b).norm() / (b.norm() + 1e-30))


@cuda
def test_qformer_golden_fp32():
    import capk
    from capk.models.qformer import QFormer
    z = np.load(GOLD, allow_pickle=False)
    D, Q, H, S, B = [int(x) for x in z["meta/dims"]]
    m = QFormer(query_dim=D, vision_dim=D, num_queries=Q, num_layers=2, num_heads=H, dropout=0.1)
    sd = {k[3:]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("p0/")}
    m.load_state_dict(sd, strict=True)
    capk.prepare(m, "cuda", "fp32")
    m.eval()
    feats = torch.from_numpy(z["in/features"]).cuda().requires_grad_(True)
    out = m(feats)["queries"]
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["out/queries"], rtol=1e-4, atol=1e-5)
    out.backward(torch.from_numpy(z["in/grad_out"]).cuda())
    np.testing.assert_allclose(feats.grad.cpu().numpy(), z["out/dfeatures"], rtol=2e-4,
                               atol=2e-4 * float(np.abs(z["out/dfeatures"]).max()))
    for n, p in m.named_parameters():
        ref = z["grad/" + n]
        np.testing.assert_allclose(p._capk_grad.cpu().numpy().reshape(ref.shape), ref, rtol=2e-4,
                                   atol=2e-4 * float(np.abs(ref).max()) + 1e-8, err_msg=n)


@cuda
def test_qformer_full_size_bf16_vs_oracle():
    import capk
    from capk.models.qformer import QFormer
    from oracle import encoders as oenc
    torch.manual_seed(3)
    m = QFormer()
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    capk.prepare(m, "cuda", "bf16")
    m.eval()
    B, N, D = 4, 197, 768
    seq = torch.randn(B, N, D)
    feats = seq[:, 1:]  # ViT features: a strided view skipping the CLS rows
    got = m(seq.cuda().bfloat16()[:, 1:])["queries"]
    ref = oenc.qformer(sd, feats.bfloat16().float(), 2, 8)
    assert got.shape == (B, 32, D)
    assert _rel(got, ref) < 3e-2, _rel(got, ref)


@cuda
def test_captioning_model_with_q_former_trains_and_generates():
    import capk
    from capk import config as C
    from capk.models import captioning_model as cm
    from capk.train import CapkAdamW, CombinedLoss
    torch.manual_seed(4)
    cfg = C.Config()
    cfg.model.encoder = C.EncoderConfig(encoder_type="vit")
    cfg.model.decoder = C.DecoderConfig(decoder_type="transformer", hidden_dim=768, num_layers=2, num_heads=8)
    cfg.model.use_q_former = True
    cfg.model.vocab_size, cfg.model.pad_token_id = 50257, 50256
    cfg.model.bos_token_id = cfg.model.eos_token_id = 50256
    model = cm.ImageCaptioningModel(cfg)
    store = capk.prepare(model, "cuda", "bf16")
    opt = CapkAdamW(store, lr=1e-4)
    model.train()
    g = torch.Generator(device="cuda").manual_seed(0)
    images = torch.randn(4, 3, 224, 224, device="cuda", generator=g)
    caps = torch.randint(0, 50256, (4, 12), device="cuda", generator=g)
    losses = []
    for _ in range(3):
        loss = CombinedLoss(50256)(logits=model(images=images, captions=caps)["logits"], targets=caps)["total_loss"]
        loss.backward()
        for n in ("q_former.query_tokens", "q_former.decoder.layers.1.multihead_attn.in_proj_weight",
                  "encoder.model.layers.11.mlp.fc2.weight"):
            gr = dict(model.named_parameters())[n]._capk_grad
            assert torch.isfinite(gr).all() and float(gr.abs().sum()) > 0, n
        opt.step()
        losses.append(float(loss))
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses
    model.eval()
    with torch.no_grad():
        ids, _ = model.generate(images=images, max_length=6)
    assert ids.shape[0] == 4
