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
