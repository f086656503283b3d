"""Self-critical sequence training.

Restates CaptioningTrainer._train_reinforcement_learning / _sample_captions /
_calculate_rewards (src/train/trainer.py:319-484) with the SURVEY fixes:

* D8  — the advantage is per sample (r_sample - r_baseline) and the loss is the mean of
        -logp * advantage over the sampled tokens up to and including the first EOS;
* D9  — the reward is a per-sample CIDEr-D on token ids, scored by the host C++ scorer
        (capk.cider -> csrc/cider.cpp; pycocoevalcap is absent: parity unpinned vs it,
        pinned by known answers and the oracle/cider.py restatement);
* sampling — the reference re-runs the full decoder on the prefix every step and keeps the
        log-prob graph; here the sampler runs the KV-cached decode step without a graph
        (softmax + inverse-CDF kernel, counter-based uniforms) and ONE teacher-forced
        forward + backward over the sampled sequence produces the same log-probabilities
        and gradients.  Sampling and scoring both use generate()'s attention semantics
        (no key-padding mask inside a generated prefix).
* baseline — model.generate (greedy for the Transformer decoder, beam-4 for GPT-2, the
        reference's greedy loop from start token 1 for the LSTM decoder), reusing the encoder
        features of the step instead of re-encoding the images.
* LSTM decoder — the reference sampler reads ``decoder.bos_token_id`` / ``eos_token_id``,
        which its LSTMDecoder does not define (``--use_rl --decoder_type lstm`` raises there);
        here build_decoder gives the LSTM decoder the model's ids and the sampler runs the
        incremental LSTM step (capk.models.lstm.LSTMStepRunner): the reference's full
        re-decode of the prefix computes the same last-position logits (no dropout in the
        sampler, the hidden state of a prefix does not depend on later tokens).
"""
import os
import threading
import time

import weakref

import numpy as np
import torch

from .. import ops
from ..cider import cider_d
from .losses import _padded_base

EOS_CHECK_EVERY = 4  # sampled steps between host checks of the all-EOS stop rule
# the baseline search runs on a side stream (its own host thread) concurrently with the
# sampler: both decode loops are chains of small latency-bound launches that leave most CUs
# idle (CAPK_SCST_CONCURRENT=0: one after the other)
CONCURRENT = os.environ.get("CAPK_SCST_CONCURRENT", "1") != "0"
_SIDE = {}
_WARM = weakref.WeakKeyDictionary()  # decoder -> set of (device, batch, max_length, baseline kwargs) already run


def _side_stream(dev):
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return s

PG_IGNORE = -100


def strip_special(ids, eos, pad, bos=None):
    """Token ids of a caption for scoring (tokenizer.decode(skip_special_tokens=True)):
    drop a leading bos, cut at the first eos, drop pads."""
    out = []
    seq = list(ids)
    if bos is not None and seq and seq[0] == bos:
        seq = seq[1:]
    for t in seq:
        if t == eos:
            break
        if t != pad:
            out.append(int(t))
    return out


# ------------------------------------------------------------- PG loss -------
class _PGLossFn(torch.autograd.Function):
    """loss = sum_{b,t counted} w_b * (-log p(target)) / count  (shifted like the CE)."""

    @staticmethod
    def forward(ctx, logits, targets, weights):
        B, T, V = logits.shape
        base = _padded_base(logits)
        targets = targets.contiguous()
        w = weights.float().contiguous()
        loss = ops.shifted_ce(base, targets, B, T, V, PG_IGNORE, want_loss=True, row_weight=w)
        ctx.save_for_backward(targets, w)
        ctx.base = base
        ctx.dims = (B, T, V)
        return loss[0]

    @staticmethod
    def backward(ctx, dloss):
        targets, w = ctx.saved_tensors
        B, T, V = ctx.dims
        base = ctx.base
        ctx.base = None
        dbase = torch.empty_like(base)
        ops.shifted_ce(base, targets, B, T, V, PG_IGNORE, want_loss=False, dlogits=dbase,
                       grad_scale=dloss.reshape(1).float().contiguous(), row_weight=w)
        return dbase[:, :V].view(B, T, V), None, None


def pg_targets(sample_ids, eos):
    """Sampled ids [B, T'] (position 0 = bos) -> CE targets where every token after the first
    EOS is ignored (the EOS itself is scored) — SURVEY D8 masking."""
    tgt = sample_ids.clone()
    is_eos = sample_ids[:, 1:] == eos
    after = torch.cumsum(is_eos.int(), 1) - is_eos.int() > 0  # strictly after the first eos
    tgt[:, 1:][after] = PG_IGNORE
    return tgt


def policy_gradient_loss(logits, sample_ids, advantages, eos):
    return _PGLossFn.apply(logits, pg_targets(sample_ids, eos), advantages)


# ------------------------------------------------------------- sampling ------
@torch.no_grad()
def sample_captions(decoder, encoder_features, max_length, seed, check_every=EOS_CHECK_EVERY):
    """_sample_captions (trainer.py:383-438): start from bos, sample from
    softmax(last logits), stop after the first step whose sampled tokens are ALL EOS
    (trainer.py:435-436).  Returns sampled ids [B, T'+1] (bos first) and the log-probs of
    the sampled tokens [B, T'].

    The stop rule is evaluated on the device every step (one flag per step) and read by
    the host only every `check_every` steps: the uniforms are counter-based per
    (seed, step, row), so steps sampled past the stop are simply cut off and the result
    equals a per-step check, without a host sync per token."""
    from .. import graphs
    from ..models.decoders import GPT2Decoder, LSTMDecoder, TransformerDecoder
    use_graphs = graphs.active()
    if isinstance(decoder, LSTMDecoder):
        from ..models.lstm import LSTMStepRunner
        feats, pooled = encoder_features["features"], encoder_features["pooled_features"]
        make = lambda: LSTMStepRunner(decoder, feats, pooled, 1, max_length)  # noqa: E731
        src = pooled
        use_graphs = False  # the runner's hoisted key/value buffers are built per call (eager loop)
    elif isinstance(decoder, TransformerDecoder):
        from ..models.transformer import KVDecodeRunner, _mem_geometry
        feats = encoder_features["features"]
        make = lambda: KVDecodeRunner(decoder, feats, 1, max_length)  # noqa: E731
        key = ("tdec", tuple(feats.shape), _mem_geometry(feats)[1], feats.dtype, 1, max_length)
        src = feats
    elif isinstance(decoder, GPT2Decoder):
        from ..models.gpt2 import GPT2KVRunner
        pooled = encoder_features["pooled_features"]
        make = lambda: GPT2KVRunner(decoder, pooled, 1, max_length)  # noqa: E731
        key = ("gpt2", pooled.shape[0], pooled.dtype, 1, max_length)
        src = pooled
    else:
        raise TypeError(f"capk SCST sampler: unknown decoder {type(decoder).__name__}")
    if use_graphs:  # cached runner, chunks of steps replayed as HIP graphs (capk/graphs.py)
        runner = graphs.runner_for(decoder, ("sample",) + key, make)
        runner.load(src)
        if runner.warm:
            ids, logp, steps = graphs.sample_generate(runner, decoder, max_length, seed, check_every)
            return ids[:, :steps + 1].clone(), logp[:steps].t().clone()
        runner.warm = True
    else:
        runner = make()
    B, dev = src.shape[0], src.device
    ids = torch.empty(B, max_length, dtype=torch.long, device=dev)
    ids[:, 0] = decoder.bos_token_id
    logp = torch.empty(max_length - 1, B, dtype=torch.float32, device=dev)
    alleos = torch.zeros(max_length - 1, dtype=torch.bool, device=dev)
    cur = ids[:, 0].contiguous()
    steps = max_length - 1
    for t in range(max_length - 1):
        logits = runner.step(t + 1, cur, None)
        nxt = torch.empty(B, dtype=torch.long, device=dev)
        ops.sample_rows(logits, decoder.vocab_size, seed, t, nxt, logp[t])
        ids[:, t + 1] = nxt
        cur = nxt
        alleos[t] = (nxt == decoder.eos_token_id).all()
        if (t + 1) % check_every == 0 or t == max_length - 2:
            hit = torch.nonzero(alleos[:t + 1])
            if hit.numel():
                steps = int(hit[0, 0]) + 1
                break
    T = steps + 1
    return ids[:, :T], logp[:steps].t()


class _Phases:
    """Per-phase GPU time of an SCST update (HIP events on the compute stream) plus the host
    time of the CIDEr-D scoring; ``times`` (dict) accumulates milliseconds per phase."""

    def __init__(self, times):
        self.times = times
        self.marks = []

    def mark(self, name):
        if self.times is None:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.marks.append((name, ev))

    def close(self, host_ms):
        if self.times is None:
            return
        self.marks[-1][1].synchronize()
        for (_, e0), (name, e1) in zip(self.marks, self.marks[1:]):
            self.times[name] = self.times.get(name, 0.0) + e0.elapsed_time(e1)
        self.times["cider_host"] = self.times.get("cider_host", 0.0) + host_ms


def scst_step(model, images, references, optimizer, lr, seed, max_length=20, baseline_kwargs=None, bucketer=None,
              phase_times=None):
    """One SCST update (trainer.py:338-381): encoder forward, sampled captions, baseline
    captions (model.generate), per-sample CIDEr-D rewards, loss = masked mean of
    -logp * (r_sample - r_baseline), backward, AdamW step.  references: per image a list
    of token-id lists.  `seed` keys the sampler's uniforms: pass a fresh value per update
    (the trainer derives it from its step counter) or every update reuses the same draws.
    `lr` = None uses the optimizer's scheduled rate.  Returns (loss, mean sample reward,
    mean baseline reward).

    The rewards are needed only by the loss: the sampled ids are copied to pinned host memory
    right after sampling and scored on a host thread while the GPU runs the baseline search;
    the baseline ids likewise while it runs the teacher-forced forward.  ``phase_times``
    (dict, optional) accumulates the GPU milliseconds of each phase (encoder, sample,
    baseline, forward, loss_backward, optimizer) and the host scoring time."""
    dec = model.decoder
    ph = _Phases(phase_times)
    ph.mark("start")
    enc = model.encoder(images)
    ph.mark("encoder")
    enc_nograd = {k: (v.detach() if torch.is_tensor(v) else v) for k, v in enc.items()}
    # Concurrent decode loops once this decoder's runners, graphs and fp8 weight copies exist
    # (the first update runs them one after the other: lazily created state is never shared
    # between the two threads); the stale fp8 copies are re-quantised here, before the fork.
    dev = next(v.device for v in enc_nograd.values() if torch.is_tensor(v))  # (images may be None: a stub encoder)
    # keyed on everything that selects a decode runner / graph / fp8 copy (a new batch size or
    # max_length builds new ones), held weakly so a new decoder never inherits a dead one's entry
    key = (dev, int(enc_nograd["features"].shape[0]) if torch.is_tensor(enc_nograd.get("features")) else None,
           int(max_length), repr(sorted((baseline_kwargs or {}).items())))
    concurrent = CONCURRENT and dev.type == "cuda" and key in _WARM.get(dec, ())
    side_out = {}
    if concurrent:
        ops.FP8.refresh()
        main = torch.cuda.current_stream()
        side = _side_stream(dev)
        side.wait_stream(main)

        def run_baseline():
            try:
                with torch.cuda.stream(side), torch.no_grad():
                    side_out["ids"] = dec.generate(enc_nograd, max_length, **(baseline_kwargs or {}))[0]
            except BaseException as ex:  # re-raised on the main thread
                side_out["err"] = ex

        th_base = threading.Thread(target=run_baseline)
        th_base.start()
    ids, _ = sample_captions(dec, enc_nograd, max_length, seed)
    ph.mark("sample")
    if concurrent:
        th_base.join()
        if "err" in side_out:
            raise side_out["err"]
        main.wait_stream(side)
        side_out["ids"].record_stream(main)
    eos, pad, bos = dec.eos_token_id, dec.pad_token_id, dec.bos_token_id
    refs = [[list(x) for x in rs] for rs in references]
    host = {"ms": 0.0}

    def score_async(dev_ids):
        """copy ids to pinned memory behind the work queued so far and score them on a host
        thread (the C++ scorer releases the GIL) while the GPU runs what comes next"""
        h = torch.empty(dev_ids.shape, dtype=dev_ids.dtype, pin_memory=True)
        h.copy_(dev_ids, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        out = {}

        def run():
            ev.synchronize()
            t0 = time.perf_counter()
            out["r"] = cider_d([strip_special(r, eos, pad, bos) for r in h.tolist()], refs)
            host["ms"] += (time.perf_counter() - t0) * 1e3

        th = threading.Thread(target=run)
        th.start()
        return th, out

    th_s, out_s = score_async(ids)  # the samples are scored during the baseline search
    if concurrent:
        base_ids = side_out["ids"]
    else:
        with torch.no_grad():
            base_ids, _ = dec.generate(enc_nograd, max_length, **(baseline_kwargs or {}))
    ph.mark("baseline")
    th_b, out_b = score_async(base_ids)  # the baselines during the teacher-forced forward
    from ..models.decoders import GPT2Decoder, LSTMDecoder
    if isinstance(dec, GPT2Decoder):
        logits = dec.forward_logits(enc["pooled_features"], ids, use_pad_mask=False)
    elif isinstance(dec, LSTMDecoder):
        logits, _ = dec.forward_logits(enc["features"], enc["pooled_features"], ids)
    else:
        logits, _ = dec.forward_logits(enc["features"], ids, use_pad_mask=False)
    ph.mark("forward")
    th_s.join()
    th_b.join()
    r_s, r_b = out_s["r"], out_b["r"]
    host_ms = host["ms"]
    adv_h = torch.from_numpy((r_s - r_b).astype(np.float32)).pin_memory()
    adv = adv_h.to(ids.device, non_blocking=True)
    loss = policy_gradient_loss(logits, ids, adv, eos)
    loss.backward()
    if bucketer is not None:  # DP: rewards are rank-local, gradients are averaged
        bucketer.finish()
    ph.mark("loss_backward")
    optimizer.step(lr=lr)
    ph.mark("optimizer")
    ph.close(host_ms)
    _WARM.setdefault(dec, set()).add(key)
    return loss.detach(), float(np.mean(r_s)), float(np.mean(r_b))
