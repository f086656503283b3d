"""Oracle restatement of HF beam search.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates transformers 5.15 ``GenerationMixin._beam_search`` and helpers
(transformers/generation/utils.py: _get_top_k_continuations, _get_running_beams_for_next_iteration,
_update_finished_beams, _check_early_stop_heuristic, _beam_search_has_unfinished_sequences)
for a decoder-only prompt of length 1 with MaxLength + EOS stopping criteria — the
path the reference reaches through ``GPT2Decoder.generate`` (src/models/decoders.py:645-654)
and, per SURVEY D16, the beam-5 semantics applied to every decoder via a per-step
logits callback ``logits_fn(flat_sequences[B*k, cur_len]) -> [B*k, V]``.
"""
import torch


def beam_search(logits_fn, batch_size, num_beams, max_length, bos, eos, pad=None, length_penalty=1.0,
                early_stopping=False, vocab_size=None, prompt=None):
    """HF semantics: prompt of length 1 (``bos`` for every image, or ``prompt[B, 1]``),
    ``eos`` single id, ``pad`` fills unfinished tails (pad or eos, utils.py:3323)."""
    # transformers/generation/utils.py:3208-3535 (_beam_search); helper line refs below
    k = num_beams
    eos_t = torch.tensor([eos])
    beams_to_keep = max(2, 1 + 1) * k
    top_num_beam_mask = torch.cat([torch.ones(k, dtype=torch.bool), torch.zeros(beams_to_keep - k, dtype=torch.bool)])
    fill = pad if pad is not None else eos
    cur_len = 1
    prompt_len = 1
    running_sequences = torch.full((batch_size, k, max_length), fill, dtype=torch.int64)
    running_sequences[:, :, 0] = (prompt.view(batch_size, 1) if prompt is not None else bos)
    sequences = running_sequences.clone()
    running_beam_scores = torch.zeros(batch_size, k)
    running_beam_scores[:, 1:] = -1e9
    beam_scores = torch.full((batch_size, k), -1e9)
    is_sent_finished = torch.zeros(batch_size, k, dtype=torch.bool)
    unsat = torch.ones(batch_size, 1, dtype=torch.bool)
    running_beam_indices = torch.full((batch_size, k, max_length - cur_len), -1, dtype=torch.int32)
    beam_indices = running_beam_indices.clone()

    def gather(t, idx):
        while idx.dim() < t.dim():
            idx = idx.unsqueeze(-1)
        return torch.gather(t, 1, idx.expand(*idx.shape[:2], *t.shape[2:]))

    while True:
        flat = running_sequences[:, :, :cur_len].reshape(batch_size * k, cur_len)
        logits = logits_fn(flat).float()
        V = logits.shape[-1] if vocab_size is None else vocab_size
        log_probs = torch.log_softmax(logits, dim=-1).view(batch_size, k, V)
        log_probs = log_probs + running_beam_scores[:, :, None]
        log_probs = log_probs.reshape(batch_size, k * V)
        # _get_top_k_continuations (utils.py:3077-3129)
        topk_log_probs, topk_indices = torch.topk(log_probs, k=beams_to_keep)
        cur_beam = topk_indices // V
        topk_running_beam_indices = gather(running_beam_indices, cur_beam)
        topk_running_sequences = gather(running_sequences, cur_beam)
        topk_ids = topk_indices % V
        topk_running_sequences[:, :, cur_len] = topk_ids
        batch_offset = torch.arange(batch_size).view(-1, 1) * k
        topk_running_beam_indices[:, :, cur_len - prompt_len] = (cur_beam + batch_offset).to(torch.int32)
        # stopping criteria: max length, eos
        hits = torch.isin(topk_ids, eos_t) | (cur_len + 1 >= max_length)
        # _get_running_beams_for_next_iteration (utils.py:3131-3151)
        topk_running_log_probs = topk_log_probs + hits.float() * -1.0e9
        nxt = torch.topk(topk_running_log_probs, k=k)[1]
        running_sequences = gather(topk_running_sequences, nxt)
        running_beam_scores = gather(topk_running_log_probs, nxt)
        running_beam_indices = gather(topk_running_beam_indices, nxt)
        # _update_finished_beams (utils.py:3153-3206)
        just_finished = hits & top_num_beam_mask[None, :]
        scored = topk_log_probs / ((cur_len + 1 - prompt_len) ** length_penalty)
        full = torch.all(is_sent_finished, dim=-1, keepdim=True) & (early_stopping is True)
        scored = scored + full.float() * -1.0e9
        scored = scored + (~unsat).float() * -1.0e9
        scored = scored + (~just_finished).float() * -1.0e9
        m_seq = torch.cat([sequences, topk_running_sequences], 1)
        m_sc = torch.cat([beam_scores, scored], 1)
        m_bi = torch.cat([beam_indices, topk_running_beam_indices], 1)
        m_fin = torch.cat([is_sent_finished, just_finished], 1)
        top = torch.topk(m_sc, k=k)[1]
        sequences, beam_scores = gather(m_seq, top), gather(m_sc, top)
        beam_indices, is_sent_finished = gather(m_bi, top), gather(m_fin, top)
        cur_len += 1
        # _check_early_stop_heuristic (utils.py:3008-3053)
        if early_stopping == "never" and length_penalty > 0.0:
            best_len = max_length - prompt_len
        else:
            best_len = cur_len - prompt_len
        best_running = running_beam_scores[:, :1] / (best_len ** length_penalty)
        worst_fin = torch.where(is_sent_finished, torch.min(beam_scores, dim=1, keepdim=True)[0],
                                torch.tensor(-1.0e9))
        unsat = unsat & torch.any(best_running > worst_fin, dim=-1, keepdim=True)
        # _beam_search_has_unfinished_sequences (utils.py:3055-3075; batch-global, like HF)
        improvement_possible = bool(torch.any(unsat))
        exists_open_beam = not (bool(torch.all(is_sent_finished)) and early_stopping is True)
        valid_continuations = not bool(torch.all(hits))
        if not (improvement_possible and exists_open_beam and valid_continuations):
            break
    # 5. outputs: best finished beam per image, cropped to the longest generated length
    best_bi = beam_indices[:, 0, :]
    max_gen = int(((best_bi + 1).bool()).sum(dim=1).max())
    out_len = prompt_len + max_gen
    return {"sequences": sequences[:, 0, :out_len], "sequences_scores": beam_scores[:, 0],
            "beam_indices": best_bi[:, :max_gen], "steps": cur_len - prompt_len,
            "all_sequences": sequences, "all_scores": beam_scores, "is_sent_finished": is_sent_finished}


def greedy_search(logits_fn, batch_size, max_length, eos, pad=None, prompt=None, bos=None):
    """HF ``generate(num_beams=1, do_sample=False)`` (transformers 5.15 GenerationMixin._sample
    with greedy selection, transformers/generation/utils.py): next = argmax(last logits);
    with an eos id, finished rows emit ``pad`` (``next * unfinished + pad * (1 - unfinished)``);
    a row finishes on eos; the loop stops when every row finished or the length reached
    max_length (prompt of length 1 included).  Returns sequences [B, <= max_length]."""
    fill = pad if pad is not None else eos
    seqs = (prompt.view(batch_size, 1) if prompt is not None else torch.full((batch_size, 1), bos)).long()
    unfinished = torch.ones(batch_size, dtype=torch.long)
    while seqs.shape[1] < max_length:
        nxt = logits_fn(seqs).float().argmax(-1)
        nxt = nxt * unfinished + fill * (1 - unfinished)
        seqs = torch.cat([seqs, nxt[:, None]], 1)
        unfinished = unfinished & (nxt != eos).long()
        if unfinished.max() == 0:
            break
    return seqs
