"""CPU: pin oracle/beam.py (restated HF beam search) to HF transformers 5.15
``generate(num_beams=…)`` outputs recorded in tests/golden/beam_gpt2.npz
(oracle/gen_beam_golden.py).  Sequences and beam indices must be bit-exact,
sequence scores within fp32 rounding."""
import os

import numpy as np
import pytest
import torch

from oracle.beam import beam_search, greedy_search

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "beam_gpt2.npz")
CASES = ["ref_like_k5", "eos_k4_lp08", "eos_k5_es"]


def _gpt2(z, name):
    from transformers import GPT2Config, GPT2LMHeadModel
    cfg = GPT2Config(vocab_size=61, n_positions=32, n_embd=32, n_layer=2, n_head=2, resid_pdrop=0.0, embd_pdrop=0.0,
                     attn_pdrop=0.0, bos_token_id=0, eos_token_id=7)
    m = GPT2LMHeadModel(cfg).eval()
    pre = f"{name}/w/"
    sd = {k[len(pre):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(pre)}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected and all(k.endswith("attn.bias") or k.endswith("masked_bias") for k in missing)
    return m


@pytest.mark.parametrize("name", CASES)
def test_oracle_beam_matches_hf_generate(name):
    z = np.load(GOLD)
    B, k, L, bos, eos, es = (int(v) for v in z[f"{name}/args"])
    lp = float(z[f"{name}/length_penalty"])
    m = _gpt2(z, name)
    prompt = torch.from_numpy(z[f"{name}/input_ids"])

    def logits_fn(flat):
        full = prompt.repeat_interleave(k, 0)
        assert torch.equal(flat[:, :1], full)
        with torch.no_grad():
            return m(input_ids=flat).logits[:, -1, :]

    out = beam_search(logits_fn, B, k, L, bos=None, eos=eos, pad=eos, length_penalty=lp,
                      early_stopping=bool(es), prompt=prompt)
    assert torch.equal(out["sequences"], torch.from_numpy(z[f"{name}/sequences"]))
    assert torch.equal(out["beam_indices"], torch.from_numpy(z[f"{name}/beam_indices"]))
    np.testing.assert_allclose(out["sequences_scores"].numpy(), z[f"{name}/sequences_scores"], rtol=1e-5, atol=1e-6)


GREEDY = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "greedy_gpt2.npz")


@pytest.mark.parametrize("name", ["greedy_ref_like", "greedy_eos_pad"])
def test_oracle_greedy_matches_hf_generate(name):
    """oracle greedy_search vs HF generate(num_beams=1) (GPT2Decoder.generate(num_beams=1),
    decoders.py:645-654), tests/golden/greedy_gpt2.npz: bit-exact sequences."""
    z = np.load(GREEDY)
    B, L, bos, eos, pad = (int(v) for v in z[f"{name}/args"])
    m = _gpt2(z, name)
    prompt = torch.from_numpy(z[f"{name}/input_ids"])

    def logits_fn(seqs):
        with torch.no_grad():
            return m(input_ids=seqs).logits[:, -1, :]

    out = greedy_search(logits_fn, B, L, eos=eos, pad=pad, prompt=prompt)
    assert torch.equal(out, torch.from_numpy(z[f"{name}/sequences"]))
