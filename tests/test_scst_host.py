"""Host-side SCST pieces (CPU): CIDEr-D reward properties (pycocoevalcap is absent, so the
metric itself is parity unpinned; these pin its defining properties), EOS masking of the
policy-gradient targets, and the sampler oracle's distribution."""
import numpy as np
import torch

from capk.train.scst import cider_d, pg_targets, strip_special
from oracle import scst as oscst


def test_cider_d_properties():
    from capk.train.scst import cider_d
    refs = [[[1, 2, 3, 4, 5]], [[6, 7, 8, 9]], [[1, 2, 3, 10]]]
    same = cider_d([r[0] for r in refs], refs)
    other = cider_d([[11, 12], [13], [14, 15, 16]], refs)
    assert np.all(same > other) and np.all(other == 0.0)
    assert np.allclose(cider_d([[1, 2, 3, 4, 5]], [[[1, 2, 3, 4, 5]]]), 0.0)  # single-image corpus: idf = 0


def test_pg_targets_mask_after_first_eos():
    ids = torch.tensor([[9, 1, 2, 9, 4, 9], [9, 3, 3, 3, 3, 3]])
    t = pg_targets(ids, 9)
    assert t[0].tolist() == [9, 1, 2, 9, -100, -100]
    assert t[1].tolist() == [9, 3, 3, 3, 3, 3]
    assert strip_special([9, 1, 2, 9, 4], 9, 9, 9) == [1, 2]


def test_sampler_oracle_distribution():
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(32) * 0.8).astype(np.float32)
    toks = [oscst.sample_row(x, 5, 0, r)[0] for r in range(4000)]
    freq = np.bincount(toks, minlength=32) / 4000.0
    p = np.exp(x - x.max()) / np.exp(x - x.max()).sum()
    assert np.abs(freq - p).max() < 0.03
