"""Oracle for the CIDEr-D reward.  TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of pycocoevalcap's CiderD scorer (cider_scorer.py with the
CiderD clipping and Gaussian length penalty; called by src/evaluate/metrics.py:46-110
behind CaptioningTrainer._calculate_rewards, src/train/trainer.py:440-484) on token-id
sentences.  pycocoevalcap is not installed (and needs Java), so this restatement is
**parity unpinned** against it; it is pinned by the hand-computed known answers in
tests/test_cider.py and checks the product scorer capk.cider (csrc/cider.cpp).
Mirrors the scorer's structure line for line: precook -> compute_doc_freq ->
counts2vec -> sim -> mean over n, / #refs, x10.
"""
import math
from collections import Counter, defaultdict

import numpy as np


def precook(tokens, n=4):
    c = Counter()
    for k in range(1, n + 1):
        for i in range(len(tokens) - k + 1):
            c[tuple(tokens[i:i + k])] += 1
    return c


def cider_d(candidates, references, n=4, sigma=6.0):
    crefs = [[precook(r, n) for r in refs] for refs in references]
    df = defaultdict(float)
    for refs in crefs:  # compute_doc_freq
        for ng in set(ng for r in refs for ng in r):
            df[ng] += 1.0
    ref_len = math.log(float(len(crefs)))

    def counts2vec(cnts):
        vec = [defaultdict(float) for _ in range(n)]
        norm = [0.0] * n
        length = 0
        for ng, tf in cnts.items():
            k = len(ng) - 1
            d = math.log(max(1.0, df[ng]))
            vec[k][ng] = float(tf) * (ref_len - d)
            norm[k] += vec[k][ng] ** 2
            if k == 1:
                length += tf
        return vec, [math.sqrt(x) for x in norm], length

    def sim(vh, vr, nh, nr, lh, lr):
        delta = float(lh - lr)
        val = np.zeros(n)
        for k in range(n):
            for ng in vh[k]:
                val[k] += min(vh[k][ng], vr[k][ng]) * vr[k][ng]
            if nh[k] != 0 and nr[k] != 0:
                val[k] /= nh[k] * nr[k]
            val[k] *= math.e ** (-(delta ** 2) / (2 * sigma ** 2))
        return val

    scores = np.zeros(len(candidates))
    for i, (cand, refs) in enumerate(zip(candidates, crefs)):
        vh, nh, lh = counts2vec(precook(cand, n))
        acc = np.zeros(n)
        for r in refs:
            vr, nr, lr = counts2vec(r)
            acc += sim(vh, vr, nh, nr, lh, lr)
        scores[i] = float(np.mean(acc)) / max(len(refs), 1) * 10.0
    return scores
