"""Caption-decoder plugin surface — mirrors src/models/decoders.py.

``build_decoder(DecoderConfig, AttentionConfig, vocab_size, pad, bos, eos)`` and
``CaptionDecoder.forward(encoder_features, captions, caption_lengths, **kw) ->
{"logits": [B,T,V], ...}`` / ``.generate(encoder_features, max_length, **kw) ->
(ids, info)`` keep the reference contract (decoders.py:20-69, 659-692).
"""
from abc import ABC, abstractmethod

import torch
import torch.nn as nn

from .. import ops
from ..config import AttentionConfig, DecoderConfig, DecoderType
from .gpt2 import GPT2DecoderCore
from .lstm import LSTMDecoderCore, LSTMStepRunner, lstm_greedy
from .transformer import TransformerDecoderCore


class CaptionDecoder(nn.Module, ABC):
    """decoders.py:20-69."""

    @abstractmethod
    def forward(self, encoder_features, captions=None, caption_lengths=None, **kwargs):
        ...

    @abstractmethod
    def generate(self, encoder_features, max_length, **kwargs):
        ...


class TransformerDecoder(TransformerDecoderCore, CaptionDecoder):
    """decoders.py:317-493 on libcapk kernels."""

    def __init__(self, config: DecoderConfig, vocab_size: int, pad_token_id: int, bos_token_id: int,
                 eos_token_id: int):
        TransformerDecoderCore.__init__(self, config.hidden_dim, config.num_layers, config.num_heads,
                                        config.dropout, config.max_length, vocab_size, pad_token_id)
        self.num_layers = config.num_layers
        self.bos_token_id = bos_token_id
        self.eos_token_id = eos_token_id

    def forward(self, encoder_features, captions=None, caption_lengths=None, **kwargs):
        if captions is None:
            return self.generate(encoder_features, 50)  # decoders.py:378-380
        # D4/D5: the encoder mask is all-ones (no padded image tokens) -> memory_key_padding_mask=None
        logits, hidden = self.forward_logits(encoder_features["features"], captions)
        return {"logits": logits, "hidden_states": hidden}

    @torch.no_grad()
    def generate(self, encoder_features, max_length, num_beams=1, length_penalty=1.0, early_stopping=False,
                 **kwargs):
        """num_beams == 1: greedy decoding (decoders.py:439-493): start from bos, append
        argmax of the last position, stop when every sequence emitted eos.  Same
        arithmetic as the reference's full re-decode per step (pad mask off: no pad in a
        generated prefix).

        num_beams > 1: HF beam search semantics (the reference's
        only beam search is GPT2Decoder.generate -> GenerationMixin._beam_search,
        decoders.py:645-654) on the KV-cached decoder; returns (sequences [B, <=max_length],
        {"sequences_scores", "beam_indices"})."""
        feats = encoder_features["features"]
        B = feats.shape[0]
        if num_beams > 1:
            from .. import graphs
            from ..beam import beam_search
            from .transformer import KVDecodeRunner, _mem_geometry
            prompt = torch.full((B,), self.bos_token_id, dtype=torch.long, device=feats.device)
            kw = dict(pad_token_id=self.pad_token_id, length_penalty=length_penalty, early_stopping=early_stopping,
                      vocab_size=self.vocab_size)
            if graphs.active():  # cached runner, steps replayed as HIP graphs (capk/graphs.py)
                key = ("tdec", tuple(feats.shape), _mem_geometry(feats)[1], feats.dtype, num_beams, max_length)
                runner = graphs.runner_for(self, key, lambda: KVDecodeRunner(self, feats, num_beams, max_length))
                runner.load(feats)
                out = graphs.beam_generate(runner, B, num_beams, max_length, prompt, self.eos_token_id, **kw)
            else:
                runner = KVDecodeRunner(self, feats, num_beams, max_length)
                out = beam_search(runner.step, B, num_beams, max_length, prompt, self.eos_token_id, **kw)
            return out["sequences"], {"sequences_scores": out["sequences_scores"],
                                      "beam_indices": out["beam_indices"]}
        # greedy on the KV-cached decode step: the same per-position arithmetic as the
        # reference's full re-decode of the prefix (causal attention), argmax kernel
        from .transformer import KVDecodeRunner
        from .. import ops
        runner = KVDecodeRunner(self, feats, 1, max_length)
        ids = torch.empty(B, max_length, dtype=torch.long, device=feats.device)
        ids[:, 0] = self.bos_token_id
        cur = ids[:, 0].contiguous()
        T = 1
        for t in range(max_length - 1):
            logits = runner.step(t + 1, cur, None)
            nxt = torch.empty(B, dtype=torch.long, device=feats.device)
            ops.argmax_rows(logits, self.vocab_size, nxt)
            ids[:, t + 1] = nxt
            cur = nxt
            T = t + 2
            if bool((nxt == self.eos_token_id).all()):
                break
        return ids[:, :T], {}


class LSTMDecoder(LSTMDecoderCore, CaptionDecoder):
    """decoders.py:70-314 on libcapk kernels (SURVEY A6 + the attention module of A7-A10)."""

    def __init__(self, config: DecoderConfig, attention_config: AttentionConfig, vocab_size: int, pad_token_id: int,
                 embedding_dim: int = None):
        LSTMDecoderCore.__init__(self, config, attention_config, vocab_size, pad_token_id, embedding_dim)
        self.max_length = config.max_length
        # the reference LSTMDecoder keeps no bos/eos ids, so its SCST sampler
        # (trainer.py:404-407, 435) cannot run it; build_decoder sets the model's ids here
        self.bos_token_id = 1
        self.eos_token_id = None

    def forward(self, encoder_features, captions=None, caption_lengths=None, **kwargs):
        if captions is None:  # decoders.py:145-148 (D11: `config` restated as the decoder's own max_length)
            return self.generate(encoder_features, self.max_length)
        # caption_lengths: the reference sorts by length and unsorts afterwards (decoders.py:157-169) but builds
        # h0/c0 from the unsorted pooled features (D10); the trainer passes None -> no sort here
        logits, weights = self.forward_logits(encoder_features["features"], encoder_features["pooled_features"],
                                              captions)
        return {"logits": logits, "attention_weights": weights}

    @torch.no_grad()
    def generate(self, encoder_features, max_length, start_token_id=1, num_beams=1, length_penalty=1.0,
                 early_stopping=False, **kwargs):
        """num_beams == 1: the reference's greedy loop (decoders.py:236-314: ids[:, t] = current
        token from start_token_id, no EOS stop).  num_beams > 1 (the reference swallows it in
        **kwargs): HF beam-search semantics (capk.beam) over the LSTM step with
        prompt start_token_id and the model's eos id; returns (sequences, {"sequences_scores",
        "beam_indices"})."""
        feats, pooled = encoder_features["features"], encoder_features["pooled_features"]
        if num_beams < 2:
            return lstm_greedy(self, feats, pooled, max_length, start_token_id)
        if self.eos_token_id is None:
            raise ValueError("capk LSTMDecoder.generate(num_beams > 1) needs eos_token_id (set by build_decoder)")
        from ..beam import beam_search
        B = pooled.shape[0]
        runner = LSTMStepRunner(self, feats, pooled, num_beams, max_length)
        prompt = torch.full((B,), start_token_id, dtype=torch.long, device=pooled.device)
        out = beam_search(runner.step, B, num_beams, max_length, prompt, self.eos_token_id,
                          pad_token_id=self.pad_token_id, length_penalty=length_penalty,
                          early_stopping=early_stopping, vocab_size=self.vocab_size)
        return out["sequences"], {"sequences_scores": out["sequences_scores"], "beam_indices": out["beam_indices"]}


class GPT2Decoder(GPT2DecoderCore, CaptionDecoder):
    """decoders.py:495-656 on libcapk kernels with the D7 prefix restatement.
    Conditions on ``pooled_features`` only (patch features unused, as in the reference)."""

    def __init__(self, config: DecoderConfig, vocab_size: int = None, pad_token_id: int = None,
                 bos_token_id: int = None, eos_token_id: int = None):
        GPT2DecoderCore.__init__(self, config, vocab_size, pad_token_id, bos_token_id, eos_token_id)

    def forward(self, encoder_features, captions=None, caption_lengths=None, **kwargs):
        if captions is None:
            return self.generate(encoder_features, 50)  # decoders.py:562-564
        logits = self.forward_logits(encoder_features["pooled_features"], captions)
        # HF's labels=captions LM loss (mean over every shifted token, ignore_index -100; decoders.py:583-589);
        # the trainer uses CombinedLoss on the logits instead
        from ..train.losses import shifted_cross_entropy
        return {"logits": logits, "loss": shifted_cross_entropy(logits, captions, -100)}

    @torch.no_grad()
    def generate(self, encoder_features, max_length, num_beams=4, length_penalty=1.0, early_stopping=False,
                 **kwargs):
        """decoders.py:619-656: HF generate(num_beams, max_length, bos/eos/pad) from a
        one-token bos prompt with the image prefix as cache (D7) -> HF beam search
        semantics on the KV-cached decoder.  Returns (sequences, info)."""
        if num_beams < 2:
            return _gpt2_greedy(self, encoder_features["pooled_features"], max_length), {}
        from .. import graphs
        from ..beam import beam_search
        from .gpt2 import GPT2KVRunner
        pooled = encoder_features["pooled_features"]
        B = pooled.shape[0]
        prompt = torch.full((B,), self.bos_token_id, dtype=torch.long, device=pooled.device)
        kw = dict(pad_token_id=self.pad_token_id, length_penalty=length_penalty, early_stopping=early_stopping,
                  vocab_size=self.vocab_size)
        if graphs.active():  # cached runner, steps replayed as HIP graphs (capk/graphs.py)
            key = ("gpt2", B, pooled.dtype, num_beams, max_length)
            runner = graphs.runner_for(self, key, lambda: GPT2KVRunner(self, pooled, num_beams, max_length))
            runner.load(pooled)
            out = graphs.beam_generate(runner, B, num_beams, max_length, prompt, self.eos_token_id, **kw)
        else:
            runner = GPT2KVRunner(self, pooled, num_beams, max_length)
            out = beam_search(runner.step, B, num_beams, max_length, prompt, self.eos_token_id, **kw)
        return out["sequences"], {"sequences_scores": out["sequences_scores"], "beam_indices": out["beam_indices"]}


def _gpt2_greedy(self, pooled, max_length):
    """HF generate(num_beams=1, do_sample=False) from the one-token bos prompt
    (GenerationMixin._sample with greedy selection, transformers/generation/utils.py):
    next = argmax(last logits); rows that already emitted eos get pad_token_id
    (next * unfinished + pad * (1 - unfinished)); stop when every row has finished or the
    sequence reached max_length (prompt included).  KV-cached decode, argmax on the device."""
    from .gpt2 import GPT2KVRunner
    B, dev = pooled.shape[0], pooled.device
    runner = GPT2KVRunner(self, pooled, 1, max_length)
    ids = torch.empty(B, max_length, dtype=torch.long, device=dev)
    ids[:, 0] = self.bos_token_id
    unfinished = torch.ones(B, dtype=torch.bool, device=dev)
    pad = self.pad_token_id if self.pad_token_id is not None else self.eos_token_id
    cur = ids[:, 0].contiguous()
    T = 1
    for t in range(1, max_length):
        logits = runner.step(t, cur, None)
        nxt = torch.empty(B, dtype=torch.long, device=dev)
        ops.argmax_rows(logits, self.vocab_size, nxt)
        nxt = torch.where(unfinished, nxt, torch.full_like(nxt, pad))
        ids[:, t] = nxt
        cur = nxt
        T = t + 1
        unfinished &= nxt != self.eos_token_id
        if not bool(unfinished.any()):
            break
    return ids[:, :T]


def build_decoder(config: DecoderConfig, attention_config: AttentionConfig, vocab_size: int, pad_token_id: int,
                  bos_token_id: int, eos_token_id: int) -> CaptionDecoder:
    """decoders.py:659-692 (with D2: string types accepted; D3: attention hidden_dim filled)."""
    dt = config.decoder_type if isinstance(config.decoder_type, DecoderType) else DecoderType(config.decoder_type)
    attention_config.hidden_dim = config.hidden_dim
    if dt == DecoderType.TRANSFORMER:
        return TransformerDecoder(config, vocab_size, pad_token_id, bos_token_id, eos_token_id)
    if dt == DecoderType.GPT2:
        return GPT2Decoder(config, vocab_size, pad_token_id, bos_token_id, eos_token_id)
    if dt == DecoderType.LSTM:
        d = LSTMDecoder(config, attention_config, vocab_size, pad_token_id)
        d.bos_token_id, d.eos_token_id = bos_token_id, eos_token_id
        return d
    raise ValueError(f"Unsupported decoder type: {config.decoder_type}")
