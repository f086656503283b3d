"""Device beam search driver.

``beam_search(step_fn, ...)`` runs transformers 5.15 ``GenerationMixin._beam_search``
semantics (transformers/generation/utils.py:3208-3535; the search behind
``GPT2Decoder.generate``, src/models/decoders.py:645-654, applied to every decoder
per SURVEY D16) with all per-step work on the GPU: the decoder's ``step_fn`` produces
logits for every running beam, ``capk_beam_step`` (csrc/beam.hip) does
log-softmax + running-score + top-2k + bookkeeping and emits the next tokens and the
KV-cache reorder indices.  The host only reads three flag words per step (HF's
batch-global stopping rule).

``step_fn(cur_len, ids, reorder) -> logits`` receives the tokens at position
``cur_len - 1`` for all ``B*k`` beams (int64 [B*k]) and, after the first step, the
int32 [B*k] reorder index (row r continues from row reorder[r]) that must be applied to
its cache *before* consuming ``ids``; it returns [B*k, ld] logits (V valid columns,
unit column stride).
"""
import torch

from . import _lib
from ._lib import check
from .ops import _need_gpu, _stream, dtype_code


def _lp_div(n, length_penalty):
    # HF: python int ** python float -> python float; dividing an fp32 tensor converts it to fp32
    return float(n ** length_penalty)


def beam_search(step_fn, batch_size, num_beams, max_length, prompt, eos_token_id, pad_token_id=None,
                length_penalty=1.0, early_stopping=False, vocab_size=None):
    """Returns dict(sequences [B, out_len] int64, sequences_scores [B] fp32, beam_indices [B, out_len-1] int32,
    all_sequences [B, k, L], all_scores [B, k], steps).  ``prompt``: int64 [B] device tensor (prompt length 1)."""
    L_ = _lib.load()
    B, k, L = batch_size, num_beams, max_length
    _need_gpu(prompt)
    dev = prompt.device
    nbytes = L_.capk_beam_state_bytes(B, k, L)
    if nbytes == 0:
        raise _lib.CapkError("capk beam_search: bad sizes")
    state = torch.empty(int(nbytes), dtype=torch.uint8, device=dev)
    fill = pad_token_id if pad_token_id is not None else eos_token_id  # utils.py:3323
    prompt = prompt.to(torch.int64).contiguous()
    st = _stream()
    check(L_.capk_beam_init(B, k, L, prompt.data_ptr(), int(fill), state.data_ptr(), int(nbytes), st),
          "capk_beam_init")
    es_code = 1 if early_stopping is True else (2 if early_stopping == "never" else 0)
    ids = prompt.repeat_interleave(k)
    reorder = torch.empty(B * k, dtype=torch.int32, device=dev)
    next_ids = torch.empty(B * k, dtype=torch.int64, device=dev)
    flags = torch.zeros(3, dtype=torch.int32).pin_memory()
    cur_len, prompt_len = 1, 1
    first = True
    while True:
        logits = step_fn(cur_len, ids, None if first else reorder)
        first = False
        V = vocab_size or logits.shape[1]
        assert logits.stride(1) == 1 and logits.shape[0] == B * k
        fin_div = _lp_div(cur_len + 1 - prompt_len, length_penalty)
        best_len = (L - prompt_len) if (early_stopping == "never" and length_penalty > 0.0) else \
            (cur_len + 1 - prompt_len)
        best_div = _lp_div(best_len, length_penalty)
        check(L_.capk_beam_step(dtype_code(logits), B, k, L, V, logits.stride(0), logits.data_ptr(), cur_len,
                                int(eos_token_id), fin_div, best_div, es_code, state.data_ptr(), int(nbytes),
                                reorder.data_ptr(), next_ids.data_ptr(), st), "capk_beam_step")
        ids = next_ids
        next_ids = torch.empty_like(ids)
        cur_len += 1
        check(L_.capk_beam_flags(state.data_ptr(), flags.data_ptr(), st), "capk_beam_flags")
        f0, f1, f2 = (int(v) for v in flags.tolist())
        if not (f0 and not (early_stopping is True and not f1) and f2) or cur_len >= L:
            break
    seqs = torch.empty(B, k, L, dtype=torch.int64, device=dev)
    scores = torch.empty(B, k, dtype=torch.float32, device=dev)
    bidx = torch.empty(B, k, L - 1, dtype=torch.int32, device=dev)
    check(L_.capk_beam_finalize(B, k, L, state.data_ptr(), seqs.data_ptr(), scores.data_ptr(), bidx.data_ptr(), st),
          "capk_beam_finalize")
    # crop to the longest generated length of the best beams (utils.py:3513-3518)
    best_bi = bidx[:, 0, :]
    max_gen = int((best_bi >= 0).sum(dim=1).max())
    out_len = prompt_len + max_gen
    return {"sequences": seqs[:, 0, :out_len], "sequences_scores": scores[:, 0], "beam_indices": best_bi[:, :max_gen],
            "all_sequences": seqs, "all_scores": scores, "steps": cur_len - prompt_len}
