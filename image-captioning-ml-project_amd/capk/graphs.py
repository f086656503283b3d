"""HIP-graph replay of the KV-cached decode loops (beam search, SCST sampling).

One decode step of the 12-block GPT-2 is ~130 libcapk launches; issued one by one from
Python that is ~2 ms of host time per step, more than the step's GPU time at bs 256
(profiles/round2: a 179-ms config-5 SCST update spent ~75 ms with the GPU idle).  Here
the loops run as chunks of CHUNK steps, each captured once per runner geometry as a HIP
graph (torch.cuda.CUDAGraph = hipGraph on ROCm) and replayed; the host only touches the
device between chunks (HF's stop flags / the sampler's all-EOS rule).

What a replay relies on:

* runners (capk.models.gpt2.GPT2KVRunner, capk.models.transformer.KVDecodeRunner) are
  cached per (decoder, batch, beams, max_length, geometry) and re-``load``-ed in place, so
  every captured address stays valid; ``reset`` restores the cache / spare ping-pong
  order the capture saw;
* per-call inputs live in static buffers written before the replay (prompt tokens, the
  sampler seed -- read by the kernel from device memory, capk_sample_rows_dev);
* a chunk that runs past the host's stop point is harmless: the beam kernels keep a
  sticky device stop flag (csrc/beam.hip beam_rows_kernel) and leave the search state
  untouched, and the sampler's extra steps are cut off exactly as its eager loop does;
* fp8 weight copies are refreshed before every replay (ops.FP8.refresh) and never created
  or re-quantised inside a capture -- the first call of a runner runs eagerly (warm-up).

CAPK_GRAPHS=0 disables the replay (the eager loops run; results are identical).
"""
import os
import threading
from collections import OrderedDict

import torch

from . import _lib, ops
from ._lib import check

ENABLED = os.environ.get("CAPK_GRAPHS", "1") != "0"
CHUNK = 4
MAX_RUNNERS = 6
_RUNNERS = OrderedDict()
_CAPTURE_LOCK = threading.Lock()
_RUNNERS_LOCK = threading.RLock()  # the SCST sampler and the baseline-search thread share the cache


def active():
    return ENABLED and torch.cuda.is_available()


def runner_for(m, key, make):
    """The cached runner of decoder `m` for `key` (created by `make()` on first use)."""
    k = (id(m), key)
    with _RUNNERS_LOCK:
        r = _RUNNERS.get(k)
        if r is not None and r.owner is not m:  # id() reused by a new decoder: stale entry
            del _RUNNERS[k]
            r = None
        if r is None:
            r = make()
            r.graphs, r.pool, r.warm, r.owner = {}, None, False, m
            _RUNNERS[k] = r
            while len(_RUNNERS) > MAX_RUNNERS:
                _RUNNERS.popitem(last=False)
        else:
            _RUNNERS.move_to_end(k)
        return r


def clear():
    with _RUNNERS_LOCK:
        _RUNNERS.clear()


def _host_state(runner):
    """The runner's host-side buffer roles that a chunk's Python body changes (the KV cache /
    spare ping-pong of a reordering beam step)."""
    return (getattr(runner, "cache", None), getattr(runner, "spare", None))


def _replay(runner, key, body):
    """Capture `body` (launches on the current stream) as the graph `key` of `runner` on
    first use, then replay it.  A replay runs none of the body's Python, so the host-side
    roles the body leaves behind (which buffer is the live KV cache after the chunk's
    reorders) are recorded at capture and restored after every replay: a chunk captured
    later -- e.g. by a longer search after a short one -- then sees the buffers the replayed
    chunks before it really left live."""
    ent = runner.graphs.get(key)
    if ent is None:
        # thread_local + one capture at a time: the SCST update runs the baseline search on a
        # side thread while the main thread keeps launching the sampler on its own stream
        # (capk.train.scst); two captures in flight at once are refused by the runtime
        with _CAPTURE_LOCK:
            if runner.pool is None:
                runner.pool = torch.cuda.graph_pool_handle()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=runner.pool, capture_error_mode="thread_local"):
                body()
            ent = runner.graphs[key] = (g, _host_state(runner))
    g, after = ent
    g.replay()
    if after[0] is not None:
        runner.cache, runner.spare = after


# ------------------------------------------------------------------ beam search ----
def beam_generate(runner, batch_size, num_beams, max_length, prompt, eos_token_id, pad_token_id=None,
                  length_penalty=1.0, early_stopping=False, vocab_size=None):
    """capk.beam.beam_search(runner.step, ...) with the steps replayed in graph chunks.
    Same outputs (the search state is the device's; chunks stop at HF's stopping rule)."""
    from .beam import _lp_div, beam_search
    if not runner.warm:  # first call of this runner: eager (creates every lazily built object)
        runner.warm = True
        return beam_search(runner.step, batch_size, num_beams, max_length, prompt, eos_token_id,
                           pad_token_id=pad_token_id, length_penalty=length_penalty,
                           early_stopping=early_stopping, vocab_size=vocab_size)
    L_ = _lib.load()
    B, k, L = batch_size, num_beams, max_length
    dev = prompt.device
    st = ops._stream()
    nbytes = L_.capk_beam_state_bytes(B, k, L)
    bb = getattr(runner, "beam_bufs", None)
    if bb is None:
        bb = runner.beam_bufs = {
            "state": torch.empty(int(nbytes), dtype=torch.uint8, device=dev),
            "ids": torch.empty(B * k, dtype=torch.int64, device=dev),
            "next": torch.empty(B * k, dtype=torch.int64, device=dev),
            "reorder": torch.empty(B * k, dtype=torch.int32, device=dev),
            "flags": torch.zeros(3, dtype=torch.int32).pin_memory()}
    state = bb["state"]
    fill = pad_token_id if pad_token_id is not None else eos_token_id
    prompt = prompt.to(torch.int64).contiguous()
    check(L_.capk_beam_init(B, k, L, prompt.data_ptr(), int(fill), state.data_ptr(), int(nbytes), st),
          "capk_beam_init")
    bb["ids"].copy_(prompt.repeat_interleave(k))
    runner.reset()
    ops.FP8.refresh()
    es_code = 1 if early_stopping is True else (2 if early_stopping == "never" else 0)
    V = vocab_size

    def one(cur_len):
        logits = runner.step(cur_len, bb["ids"], None if cur_len == 1 else bb["reorder"])
        fin_div = _lp_div(cur_len, length_penalty)
        best_len = (L - 1) if (early_stopping == "never" and length_penalty > 0.0) else cur_len
        best_div = _lp_div(best_len, length_penalty)
        check(L_.capk_beam_step(ops.dtype_code(logits), B, k, L, V or logits.shape[1], logits.stride(0),
                                logits.data_ptr(), cur_len, int(eos_token_id), fin_div, best_div, es_code,
                                state.data_ptr(), int(nbytes), bb["reorder"].data_ptr(), bb["next"].data_ptr(),
                                ops._stream()),  # the capture stream while capturing
              "capk_beam_step")
        bb["ids"].copy_(bb["next"])

    cur_len = 1
    flags = bb["flags"]
    while cur_len < L:
        c1 = min(L, cur_len + CHUNK)
        c0 = cur_len
        _replay(runner, ("beam", c0, c1, V, int(eos_token_id), es_code, float(length_penalty)),
                lambda: [one(c) for c in range(c0, c1)])
        cur_len = c1
        check(L_.capk_beam_flags(state.data_ptr(), flags.data_ptr(), st), "capk_beam_flags")
        f0, f1, f2 = (int(v) for v in flags.tolist())
        if not (f0 and not (early_stopping is True and not f1) and f2):
            break
    seqs = torch.empty(B, k, L, dtype=torch.int64, device=dev)
    scores = torch.empty(B, k, dtype=torch.float32, device=dev)
    bidx = torch.empty(B, k, L - 1, dtype=torch.int32, device=dev)
    check(L_.capk_beam_finalize(B, k, L, state.data_ptr(), seqs.data_ptr(), scores.data_ptr(), bidx.data_ptr(), st),
          "capk_beam_finalize")
    best_bi = bidx[:, 0, :]
    max_gen = int((best_bi >= 0).sum(dim=1).max())
    out_len = 1 + max_gen
    return {"sequences": seqs[:, 0, :out_len], "sequences_scores": scores[:, 0], "beam_indices": best_bi[:, :max_gen],
            "all_sequences": seqs, "all_scores": scores}


# --------------------------------------------------------------- SCST sampling ----
def sample_generate(runner, decoder, max_length, seed, check_every):
    """capk.train.scst.sample_captions' loop with the steps replayed in graph chunks of
    `check_every` steps; returns (ids [B, max_length], logp [max_length-1, B],
    alleos [max_length-1] bool) device buffers and the number of steps run."""
    B, dev = runner.R, runner.cache.device
    sb = getattr(runner, "sample_bufs", None)
    if sb is None:
        sb = runner.sample_bufs = {
            "ids": torch.empty(B, max_length, dtype=torch.long, device=dev),
            "logp": torch.empty(max_length - 1, B, dtype=torch.float32, device=dev),
            "alleos": torch.zeros(max_length - 1, dtype=torch.bool, device=dev),
            "cur": torch.empty(B, dtype=torch.long, device=dev),
            "nxt": torch.empty(B, dtype=torch.long, device=dev),
            "seed": torch.zeros(1, dtype=torch.int32, device=dev)}
    ids, logp, alleos, cur, nxt = sb["ids"], sb["logp"], sb["alleos"], sb["cur"], sb["nxt"]
    u = int(seed) & 0xFFFFFFFF  # the kernel reads the uint32 bit pattern
    sb["seed"].fill_(u - 2 ** 32 if u >= 2 ** 31 else u)
    ids[:, 0] = decoder.bos_token_id
    cur.copy_(ids[:, 0])
    runner.reset()
    ops.FP8.refresh()
    eos = decoder.eos_token_id

    def one(t):
        logits = runner.step(t + 1, cur, None)
        ops.sample_rows(logits, decoder.vocab_size, sb["seed"], t, nxt, logp[t])
        ids[:, t + 1].copy_(nxt)
        cur.copy_(nxt)
        torch.all(nxt == eos, out=alleos[t])

    steps = max_length - 1
    t = 0
    while t < max_length - 1:
        t0, t1 = t, min(max_length - 1, t + check_every)
        _replay(runner, ("sample", t0, t1, decoder.vocab_size, int(eos)), lambda: [one(u) for u in range(t0, t1)])
        t = t1
        hit = torch.nonzero(alleos[:t])
        if hit.numel():
            steps = int(hit[0, 0]) + 1
            break
    return ids, logp, steps
