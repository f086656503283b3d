"""Oracle CPU train step for config 3 (ViT-B/16 + Transformer + MHA), used ONLY as
bench.py's reported ``cpu_baseline`` (TEST INFRASTRUCTURE; see oracle/__init__.py).

Restates CaptioningTrainer._train_epoch's fp32 branch (src/train/trainer.py:260-286):
forward (oracle.encoders / oracle.decoders), shifted CE (losses.py:236-247),
backward (torch CPU autograd), AdamW with the reference groups, scheduler step.
"""
import time

import torch

from . import decoders as odec
from . import encoders as oenc
from . import train as otrain


def _sub(p, prefix):
    return {k[len(prefix):]: v for k, v in p.items() if k.startswith(prefix)}


def make_params(state_dict):
    return {k: v.detach().float().clone().requires_grad_(True) for k, v in state_dict.items()}


def train_step(params, state, images, captions, pad, step, lr, layers=(12, 12, 16, 6, 8)):
    Le, He, P, Ld, Hd = layers
    for p in params.values():
        p.grad = None
    enc = oenc.vit_encoder(_sub(params, "encoder.model."), images, Le, He, P)
    logits = odec.transformer_decoder(_sub(params, "decoder."), enc["features"], captions, Ld, Hd, pad)
    loss = otrain.shifted_ce(logits, captions, pad)
    loss.backward()
    with torch.no_grad():
        for n, p in params.items():
            if p.grad is None:
                continue
            m, v = state.setdefault(n, (torch.zeros_like(p), torch.zeros_like(p)))
            otrain.adamw_step(p, p.grad, m, v, step, lr, 0.0 if otrain.no_decay(n) else 0.01)
    return float(loss)


def time_cpu_baseline(state_dict, batch=4, steps=2, warmup=1, pad=50256, threads=None):
    """Images/s of the oracle CPU step on a bounded sample (batch x steps)."""
    if threads:
        torch.set_num_threads(threads)
    params = make_params(state_dict)
    opt_state = {}
    g = torch.Generator().manual_seed(0)
    images = torch.randn(batch, 3, 224, 224, generator=g)
    caps = torch.randint(0, 50256, (batch, 20), generator=torch.Generator().manual_seed(1))
    for i in range(warmup):
        train_step(params, opt_state, images, caps, pad, i + 1, 5e-5)
    t0 = time.perf_counter()
    for i in range(steps):
        train_step(params, opt_state, images, caps, pad, warmup + i + 1, 5e-5)
    dt = time.perf_counter() - t0
    return batch * steps / dt, dt


def time_cpu_beam(state_dict, images=2, num_beams=5, max_length=20, threads=None, eos=50256):
    """Captions/s of the oracle CPU beam-5 path (ViT forward + oracle/beam.py over the
    decoder re-run on each prefix, as the reference's generate does) on a bounded sample."""
    import torch.nn.functional as F
    from .beam import beam_search
    if threads:
        torch.set_num_threads(threads)
    p = {k: v.detach().float() for k, v in state_dict.items()}
    dec = _sub(p, "decoder.")
    img = torch.randn(images, 3, 224, 224, generator=torch.Generator().manual_seed(7))
    t0 = time.perf_counter()
    with torch.no_grad():
        feats = oenc.vit_encoder(_sub(p, "encoder.model."), img, 12, 12, 16)["features"]
        mem = F.linear(feats, dec["visual_projection.weight"], dec["visual_projection.bias"])
        mem = mem.repeat_interleave(num_beams, 0)
        beam_search(lambda s: odec.transformer_last_logits(dec, mem, s, 6, 8), images, num_beams, max_length,
                    bos=eos, eos=eos, pad=eos)
    dt = time.perf_counter() - t0
    return images / dt, dt


def time_cpu_scst(state_dict, images=2, max_length=20, threads=None, eos=50256, refs_per_image=5):
    """Images/s of the oracle CPU SCST update for config 5 (CLIP-ViT-B/32 + GPT-2) on a
    bounded sample -- CaptioningTrainer._train_reinforcement_learning (src/train/
    trainer.py:338-381) with the SURVEY D7/D8/D9 restatements: CLIP forward (with grad),
    sampled captions (softmax sampling, the decoder re-run on each prefix as the reference's
    _sample_captions does, trainer.py:383-438), the GPT-2 baseline beam-4 generate
    (decoders.py:645-654 -> oracle/beam.py), CIDEr-D rewards (oracle/cider.py), the
    policy-gradient loss over a teacher-forced re-run, backward, AdamW."""
    from .beam import beam_search
    from .cider import cider_d
    if threads:
        torch.set_num_threads(threads)
    params = make_params(state_dict)
    enc_p, dec_p = _sub(params, "encoder.model."), _sub(params, "decoder.")
    g = torch.Generator().manual_seed(11)
    img = torch.randn(images, 3, 224, 224, generator=g)
    refs = [[torch.randint(0, eos, (int(torch.randint(8, 17, (1,), generator=g)),), generator=g).tolist()
             for _ in range(refs_per_image)] for _ in range(images)]

    def strip(seq):
        out = []
        for t in seq[1:]:
            if t == eos:
                break
            out.append(int(t))
        return out

    t0 = time.perf_counter()
    for p in params.values():
        p.grad = None
    enc = oenc.clip_encoder(enc_p, img, 12, 12, 32)
    pooled = enc["pooled_features"]
    with torch.no_grad():
        dp = {k: v.detach() for k, v in dec_p.items()}
        pd = pooled.detach()
        seqs = torch.full((images, 1), eos, dtype=torch.long)
        for _ in range(max_length - 1):
            last = odec.gpt2_decoder(dp, pd, seqs, 12, 12, eos, use_pad_mask=False)[:, -1]
            nxt = torch.distributions.Categorical(logits=last).sample()
            seqs = torch.cat([seqs, nxt[:, None]], 1)
            if bool((nxt == eos).all()):
                break
        pr = pd.repeat_interleave(4, 0)
        base = beam_search(lambda s: odec.gpt2_decoder(dp, pr, s, 12, 12, eos, use_pad_mask=False)[:, -1], images, 4,
                           max_length, bos=eos, eos=eos, pad=eos)["sequences"]
    r_s = cider_d([strip(s) for s in seqs.tolist()], refs)
    r_b = cider_d([strip(s) for s in base.tolist()], refs)
    adv = torch.tensor([a - b for a, b in zip(r_s, r_b)], dtype=torch.float32)
    logits = odec.gpt2_decoder(dec_p, pooled, seqs, 12, 12, eos, use_pad_mask=False)
    logp = torch.log_softmax(logits[:, :-1], -1).gather(2, seqs[:, 1:, None])[..., 0]
    keep = torch.ones_like(logp, dtype=torch.bool)
    for b in range(images):  # tokens up to and including the first EOS (D8)
        row = seqs[b, 1:].tolist()
        if eos in row:
            keep[b, row.index(eos) + 1:] = False
    loss = -(logp * adv[:, None] * keep).sum() / keep.sum()
    loss.backward()
    with torch.no_grad():
        opt_state = {}
        for n, p in params.items():
            if p.grad is None:
                continue
            m, v = opt_state.setdefault(n, (torch.zeros_like(p), torch.zeros_like(p)))
            otrain.adamw_step(p, p.grad, m, v, 1, 5e-5, 0.0 if otrain.no_decay(n) else 0.01)
    dt = time.perf_counter() - t0
    return images / dt, dt


def time_cpu_config2(state_dict, batch=2, steps=1, warmup=1, pad=50256, threads=None):
    """Images/s of the oracle CPU CE train step for config 2 (ResNet-101 + LSTM(768, 6 layers)
    + soft attention, train-mode BatchNorm) on a bounded sample -- the same
    _train_epoch body as time_cpu_baseline (src/train/trainer.py:218-289)."""
    from . import lstm as olstm
    if threads:
        torch.set_num_threads(threads)
    params = make_params(state_dict)
    state = {k: v.detach().clone() for k, v in state_dict.items()}
    opt_state = {}
    g = torch.Generator().manual_seed(0)
    images = torch.randn(batch, 3, 224, 224, generator=g)
    caps = torch.randint(0, pad, (batch, 20), generator=torch.Generator().manual_seed(1))

    def one(step):
        for p in params.values():
            p.grad = None
        enc = oenc.resnet_encoder(_sub(params, "encoder."), images, [256, 512, 1024, 2048], [3, 4, 23, 3],
                                  training=True, state=_sub(state, "encoder."))
        logits, _ = olstm.lstm_decoder(_sub(params, "decoder."), enc["features"], enc["pooled_features"], caps, 6,
                                       "soft")
        loss = otrain.shifted_ce(logits, caps, pad)
        loss.backward()
        with torch.no_grad():
            for n, p in params.items():
                if p.grad is None:
                    continue
                m, v = opt_state.setdefault(n, (torch.zeros_like(p), torch.zeros_like(p)))
                otrain.adamw_step(p, p.grad, m, v, step, 5e-5, 0.0 if otrain.no_decay(n) else 0.01)

    for i in range(warmup):
        one(i + 1)
    t0 = time.perf_counter()
    for i in range(steps):
        one(warmup + i + 1)
    dt = time.perf_counter() - t0
    return batch * steps / dt, dt
