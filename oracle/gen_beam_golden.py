"""Generate tests/golden/beam_gpt2.npz: HF transformers 5.15 beam search on a tiny random GPT-2.

TEST INFRASTRUCTURE ONLY.  Pins oracle/beam.py (restatement of
``GenerationMixin._beam_search``, transformers/generation/utils.py:3208-3535) to the
library the reference calls in ``GPT2Decoder.generate`` (src/models/decoders.py:645-654).
Weights are random (no network); the initializer range is raised so next-token
distributions are peaked and candidate margins are far above fp32 noise.  Each case
stores the GPT-2 weights, the generate() arguments and its outputs
(sequences, sequences_scores, beam_indices).

Run in the build container:  python oracle/gen_beam_golden.py
``python oracle/gen_beam_golden.py greedy`` writes tests/golden/greedy_gpt2.npz instead:
HF generate(num_beams=1) (greedy, the GPT2Decoder.generate(num_beams=1) path) on the same
kind of tiny models, pinning oracle/beam.py greedy_search.
"""
import os

import numpy as np
import torch
from transformers import GPT2Config, GPT2LMHeadModel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden", "beam_gpt2.npz")
GREEDY_OUT = os.path.join(ROOT, "tests", "golden", "greedy_gpt2.npz")
# (name, batch, max_length, bos, eos, pad): pad != eos exercises the finished-row fill
GREEDY_CASES = [
    ("greedy_ref_like", 4, 12, 60, 60, 60),
    ("greedy_eos_pad", 4, 14, 0, 7, 5),
]

# (name, batch, num_beams, max_length, bos, eos, length_penalty, early_stopping)
CASES = [
    ("ref_like_k5", 4, 5, 12, 60, 60, 1.0, False),   # bos == eos == pad (GPT-2 tokenizer layout)
    ("eos_k4_lp08", 3, 4, 10, 0, 7, 0.8, False),     # reference default num_beams=4, InferenceConfig lp 0.8
    ("eos_k5_es", 3, 5, 9, 0, 7, 1.0, True),        # early_stopping=True
]


def tiny_gpt2(seed):
    torch.manual_seed(seed)
    cfg = GPT2Config(vocab_size=61, n_positions=32, n_embd=32, n_layer=2, n_head=2, initializer_range=0.35,
                     resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0, bos_token_id=0, eos_token_id=7)
    m = GPT2LMHeadModel(cfg).eval()
    with torch.no_grad():  # make EOS (token 7) a frequent continuation so finished-beam merging is exercised
        m.transformer.wte.weight[7] *= 1.6
    return cfg, m


def main():
    out = {}
    for i, (name, B, k, L, bos, eos, lp, es) in enumerate(CASES):
        cfg, m = tiny_gpt2(100 + i)
        ids = torch.full((B, 1), bos, dtype=torch.long)
        # distinct prompts per row come from a different first token per image
        ids[:, 0] = torch.tensor([bos, 3, 11, 29][:B])
        with torch.no_grad():
            g = m.generate(input_ids=ids, attention_mask=torch.ones_like(ids), max_length=L, num_beams=k,
                           pad_token_id=eos, bos_token_id=bos, eos_token_id=eos, length_penalty=lp,
                           early_stopping=es, do_sample=False, return_dict_in_generate=True, output_scores=True)
        out[f"{name}/args"] = np.array([B, k, L, bos, eos, int(es)], dtype=np.int64)
        out[f"{name}/length_penalty"] = np.array(lp, dtype=np.float64)
        out[f"{name}/input_ids"] = ids.numpy()
        out[f"{name}/sequences"] = g.sequences.numpy()
        out[f"{name}/sequences_scores"] = g.sequences_scores.float().numpy()
        out[f"{name}/beam_indices"] = g.beam_indices.numpy()
        for kname, v in m.state_dict().items():
            if kname.endswith("attn.bias") or kname.endswith("masked_bias"):
                continue
            out[f"{name}/w/{kname}"] = v.float().numpy()
        print(name, g.sequences.tolist(), g.sequences_scores.tolist())
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT))


def main_greedy():
    out = {}
    for i, (name, B, L, bos, eos, pad) in enumerate(GREEDY_CASES):
        cfg, m = tiny_gpt2(200 + i)
        ids = torch.tensor([bos, 3, 11, 29][:B], dtype=torch.long)[:, None]
        with torch.no_grad():
            g = m.generate(input_ids=ids, attention_mask=torch.ones_like(ids), max_length=L, num_beams=1,
                           pad_token_id=pad, bos_token_id=bos, eos_token_id=eos, do_sample=False)
        out[f"{name}/args"] = np.array([B, L, bos, eos, pad], dtype=np.int64)
        out[f"{name}/input_ids"] = ids.numpy()
        out[f"{name}/sequences"] = g.numpy()
        for kname, v in m.state_dict().items():
            if kname.endswith("attn.bias") or kname.endswith("masked_bias"):
                continue
            out[f"{name}/w/{kname}"] = v.float().numpy()
        print(name, g.tolist())
    np.savez_compressed(GREEDY_OUT, **out)
    print("wrote", GREEDY_OUT, os.path.getsize(GREEDY_OUT))


if __name__ == "__main__":
    import sys
    main_greedy() if sys.argv[1:] == ["greedy"] else main()
