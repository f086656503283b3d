"""CIDEr-D: the SCST reward.  pycocoevalcap (and its Java tokenizer) is
absent, so the scorer is parity unpinned against it; these tests pin the restatement
by KNOWN ANSWERS computed by hand from the scorer's definition (pycocoevalcap
cider_scorer.py, CiderD variant: tf-idf n-gram vectors n = 1..4, df over the corpus
references, ref_len = ln(#images), clipped similarity min(vh, vr) * vr, Gaussian length
penalty on bigram counts with sigma 6, mean over n, / #refs, x10), then check the
product scorer (capk.cider -> csrc/cider.cpp, host C++ on threads) against the
pure-Python oracle (oracle/cider.py) on random corpora.  Host code only: no GPU."""
import math
import time

import numpy as np
import pytest

from capk.cider import cider_d
from oracle import cider as ocider

PEN1 = math.exp(-1.0 / 72.0)  # exp(-delta^2 / (2 sigma^2)), |delta| = 1, sigma = 6


@pytest.mark.parametrize("scorer", [cider_d, ocider.cider_d], ids=["capk", "oracle"])
def test_known_answer_identical_and_disjoint(scorer):
    # 2 images: L = ln 2; image 0 candidate equals its single reference -> n = 1, 2 terms
    # are 1 (n = 3, 4 have zero norms) -> mean 0.5 -> x10 = 5.0; image 1 disjoint -> 0.
    got = scorer([[1, 2], [3]], [[[1, 2]], [[4]]])
    np.testing.assert_allclose(got, [5.0, 0.0], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("scorer", [cider_d, ocider.cider_d], ids=["capk", "oracle"])
def test_known_answer_repeated_ngrams_clipping_and_length(scorer):
    # image 0: cand [5,5,5], ref [5,6].  Unigram (5): hyp tf 3 -> 3L, ref L; clipped
    # product min(3L, L) * L = L^2; |h| = 3L, |r| = sqrt(2) L -> 1 / (3 sqrt 2).
    # Bigrams (5,5) vs (5,6): no overlap.  Lengths (bigram counts) 2 vs 1 -> penalty
    # exp(-1/72).  Score = 10 * mean([1/(3 sqrt 2) * pen, 0, 0, 0]).
    got = scorer([[5, 5, 5], [7]], [[[5, 6]], [[8]]])
    want0 = 10.0 * (PEN1 / (3.0 * math.sqrt(2.0))) / 4.0
    np.testing.assert_allclose(got, [want0, 0.0], rtol=1e-12, atol=1e-12)
    assert abs(want0 - 0.58110) < 1e-4


@pytest.mark.parametrize("scorer", [cider_d, ocider.cider_d], ids=["capk", "oracle"])
def test_known_answer_multi_reference_document_frequency(scorer):
    # 3 images, L = ln 3.  Token 1 occurs in the references of images 0 and 1 -> df 2,
    # weight a = L - ln 2; every other n-gram has df <= 1 -> weight L.
    L, a = math.log(3.0), math.log(3.0) - math.log(2.0)
    cands = [[1, 2, 3], [9], [4]]
    refs = [[[1, 2, 3], [1, 2]], [[1, 9]], [[5]]]
    got = scorer(cands, refs)
    # image 0, ref [1,2,3]: identical vectors -> sims [1, 1, 1, 0]
    sim_a = [1.0, 1.0, 1.0, 0.0]
    # ref [1,2]: n=1: (a^2 + L^2) / (sqrt(a^2 + 2L^2) sqrt(a^2 + L^2)); n=2: L^2 / (sqrt2 L * L);
    # bigram lengths 2 vs 1 -> penalty exp(-1/72)
    sim_b = [math.sqrt(a * a + L * L) / math.sqrt(a * a + 2 * L * L) * PEN1, PEN1 / math.sqrt(2.0), 0.0, 0.0]
    want0 = 10.0 * (sum(sim_a) + sum(sim_b)) / 4.0 / 2.0
    # image 1: cand (9) weight L vs ref {(1): a, (9): L, (1,9): L}: L^2 / (L sqrt(a^2 + L^2));
    # bigram lengths 0 vs 1 -> penalty exp(-1/72)
    want1 = 10.0 * (L / math.sqrt(a * a + L * L) * PEN1) / 4.0
    np.testing.assert_allclose(got, [want0, want1, 0.0], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("scorer", [cider_d, ocider.cider_d], ids=["capk", "oracle"])
def test_known_answer_degenerate(scorer):
    # empty candidate: every norm is 0 -> 0; a one-image corpus has ref_len = ln 1 = 0 and
    # df = 1 -> every weight 0 -> 0 (the scorer's idf needs >= 2 images)
    np.testing.assert_allclose(scorer([[], [1, 2]], [[[1, 2]], [[1, 2]]]), [0.0, 0.0], atol=1e-15)
    np.testing.assert_allclose(scorer([[1, 2, 3, 4, 5]], [[[1, 2, 3, 4, 5]]]), [0.0], atol=1e-15)


def test_capk_matches_oracle_on_random_corpora():
    rng = np.random.default_rng(0)
    for vocab, n_img, n_ref in ((12, 64, 5), (40, 200, 3), (50257, 32, 5)):
        def sent():
            return rng.integers(0, vocab, rng.integers(0, 22)).tolist()
        cands = [sent() for _ in range(n_img)]
        refs = [[sent() for _ in range(int(rng.integers(1, n_ref + 1)))] for _ in range(n_img)]
        # also candidates that copy a reference (non-trivial overlaps at every order)
        for i in range(0, n_img, 3):
            cands[i] = list(refs[i][0])
        got = cider_d(cands, refs)
        want = ocider.cider_d(cands, refs)
        np.testing.assert_allclose(got, want, rtol=1e-11, atol=1e-12)
        np.testing.assert_array_equal(cider_d(cands, refs, threads=1), got)  # thread count does not matter


def test_capk_scorer_speed_at_scst_batch():
    """One SCST update scores 256 images x (sample + baseline) against 5 references."""
    rng = np.random.default_rng(1)
    n = 2048
    cands = [rng.integers(0, 3000, 19).tolist() for _ in range(n)]
    refs = [[rng.integers(0, 3000, int(rng.integers(8, 20))).tolist() for _ in range(5)] for _ in range(n)]
    t0 = time.perf_counter()
    s = cider_d(cands, refs)
    dt = time.perf_counter() - t0
    assert s.shape == (n,) and np.isfinite(s).all()
    assert dt < 2.0, dt
