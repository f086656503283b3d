"""HIP-graph replay of the decode loops (capk/graphs.py) against the eager loops: beam-5
generate of the Transformer decoder, beam-4 generate and SCST sampling of the GPT-2
decoder (bf16, full-size random-init weights) -- sequences, beam indices and sampled ids
bit-exact, scores / log-probs equal -- over the warm-up call, the capturing call and a
replaying call with different inputs; plus a search that stops early (EOS forced through
the output bias), where a replayed chunk runs past HF's stopping point and the sticky
device stop flag must leave the result unchanged."""
import pytest
import torch

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")


def _decoder(kind, seed=3):
    import capk
    from capk import config as C
    from capk.models.decoders import build_decoder
    torch.manual_seed(seed)
    if kind == "transformer":
        dcfg = C.DecoderConfig(decoder_type="transformer", hidden_dim=768, num_layers=6, num_heads=8)
    else:
        dcfg = C.DecoderConfig(decoder_type="gpt2", pretrained_model_name="gpt2")
    dec = build_decoder(dcfg, C.AttentionConfig(attention_type="multi_head"), 50257, 50256, 50256, 50256)
    capk.prepare(dec, "cuda", "bf16")
    dec.eval()
    return dec


def _enc(B, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return {"features": torch.randn(B, 196, 768, device="cuda", generator=g).bfloat16(),
            "pooled_features": torch.randn(B, 768, device="cuda", generator=g).bfloat16(), "attention_mask": None}


def _eager_then_graphed(fn, inputs):
    from capk import graphs
    graphs.clear()
    old = graphs.ENABLED
    try:
        graphs.ENABLED = False
        ref = [fn(x) for x in inputs]
        graphs.ENABLED = True
        got = [fn(x) for x in inputs]  # warm-up (eager), capture + replay, replay, ...
    finally:
        graphs.ENABLED = old
        graphs.clear()
    return ref, got


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if torch.is_tensor(x):
            assert x.shape == y.shape and torch.equal(x, y), (x, y)
        else:
            _same(list(x.values()) if isinstance(x, dict) else x, list(y.values()) if isinstance(y, dict) else y)


@cuda
def test_transformer_beam5_graphs_equal_eager():
    dec = _decoder("transformer")
    inputs = [_enc(3, s) for s in (1, 2, 3, 4)]

    def fn(enc):
        with torch.no_grad():
            ids, info = dec.generate(enc, 20, num_beams=5)
        return [ids.clone(), info["sequences_scores"].clone(), info["beam_indices"].clone()]

    ref, got = _eager_then_graphed(fn, inputs)
    for r, g in zip(ref, got):
        _same(r, g)


@cuda
def test_gpt2_beam4_and_sampling_graphs_equal_eager():
    from capk.train.scst import sample_captions
    dec = _decoder("gpt2")
    inputs = [(_enc(4, s), 0x5C57 + s) for s in (1, 2, 3)]

    def beam(x):
        with torch.no_grad():
            ids, info = dec.generate(x[0], 20, num_beams=4)
        return [ids.clone(), info["sequences_scores"].clone(), info["beam_indices"].clone()]

    def sample(x):
        ids, logp = sample_captions(dec, x[0], 20, x[1])
        return [ids.clone(), logp.clone()]

    for fn in (beam, sample):
        ref, got = _eager_then_graphed(fn, inputs)
        for r, g in zip(ref, got):
            _same(r, g)
    # different seeds really give different samples through the device seed
    assert not torch.equal(ref[0][0], ref[1][0])


@cuda
def test_early_stopping_search_graphs_equal_eager():
    """EOS made the likely token from the second position on (output bias): the search
    finishes after a few steps, inside a 4-step graph chunk."""
    dec = _decoder("transformer", seed=5)
    with torch.no_grad():
        dec.output_layer.bias._capk_pad_master[50256] += 12.0
    inputs = [_enc(2, s) for s in (7, 8, 9)]

    def fn(enc):
        with torch.no_grad():
            ids, info = dec.generate(enc, 20, num_beams=5)
        return [ids.clone(), info["sequences_scores"].clone(), info["beam_indices"].clone()]

    ref, got = _eager_then_graphed(fn, inputs)
    assert ref[0][0].shape[1] < 20, "the forced-EOS search should stop early"
    for r, g in zip(ref, got):
        _same(r, g)


@cuda
def test_short_search_then_full_search_graphs_equal_eager():
    """A search that stops early captures only its first chunk(s); the next, full-length
    search replays those and captures the rest.  The KV cache / spare roles the replayed
    chunks leave behind must be the ones the later capture builds on (graphs._replay
    restores them), else the later chunks read the stale cache buffer."""
    dec = _decoder("transformer", seed=5)
    bias = dec.output_layer.bias._capk_pad_master
    orig = float(bias[50256])
    # (encoder output, EOS logit boost): short, short, full, full
    inputs = [(_enc(2, 11), 12.0), (_enc(2, 12), 12.0), (_enc(2, 13), 0.0), (_enc(2, 14), 0.0)]

    def fn(x):
        enc, boost = x
        with torch.no_grad():
            bias[50256] = orig + boost
            ids, info = dec.generate(enc, 20, num_beams=5)
        return [ids.clone(), info["sequences_scores"].clone(), info["beam_indices"].clone()]

    try:
        ref, got = _eager_then_graphed(fn, inputs)
    finally:
        with torch.no_grad():
            bias[50256] = orig
    assert ref[1][0].shape[1] < 20 and ref[2][0].shape[1] == 20, [r[0].shape for r in ref]
    for r, g in zip(ref, got):
        _same(r, g)


@cuda
@pytest.mark.parametrize("kind", ["transformer", "gpt2"])
def test_history_table_equals_cache_gather(kind, monkeypatch):
    """The beam-history table (capk_attention_decode_rows: key j of hypothesis r read from
    cache row hist[r, j]) against the whole-cache reorder it replaces (CAPK_KV_GATHER=1,
    HF Cache.reorder_cache): same keys and values in the same order, so sequences, scores
    and beam indices are bit-identical, eager and graph-replayed."""
    from capk import graphs
    dec = _decoder(kind, seed=6)
    beams = 5 if kind == "transformer" else 4
    inputs = [_enc(3, s) for s in (21, 22, 23)]

    def fn(enc):
        with torch.no_grad():
            ids, info = dec.generate(enc, 20, num_beams=beams)
        return [ids.clone(), info["sequences_scores"].clone(), info["beam_indices"].clone()]

    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("CAPK_KV_GATHER", mode)
        out[mode] = _eager_then_graphed(fn, inputs)
    graphs.clear()
    for a, b in zip(out["1"], out["0"]):
        for r, g in zip(a, b):
            _same(r, g)
