"""CIDEr-D reward — host C++ scorer in libcapk (csrc/cider.cpp).

Replaces src/evaluate/metrics.py:46-110 (pycocoevalcap CiderD behind
CaptioningTrainer._calculate_rewards, src/train/trainer.py:440-484) with a per-sample
score on token ids (D9: pycocoevalcap and Java are absent, so the reference's reward
is a hard-coded 0.0; this restates the published scorer).  Parity: checked against the
pure-Python restatement oracle/cider.py and hand-computed known answers
(tests/test_cider.py); pycocoevalcap itself is unavailable — parity unpinned vs it.
"""
import ctypes

import numpy as np

from . import _lib


def _csr(seqs):
    off = np.zeros(len(seqs) + 1, dtype=np.int64)
    if seqs:
        off[1:] = np.cumsum([len(s) for s in seqs])
    tok = np.fromiter((t for s in seqs for t in s), dtype=np.int32, count=int(off[-1]))
    return np.ascontiguousarray(tok), off


def cider_d(candidates, references, n=4, sigma=6.0, threads=0):
    """candidates: list of token-id lists; references: per candidate, a list of token-id
    lists.  Returns float64 scores [len(candidates)] (x10 scale, like pycocoevalcap)."""
    if len(candidates) != len(references):
        raise ValueError(f"cider_d: {len(candidates)} candidates vs {len(references)} reference sets")
    lib = _lib.load()
    ct, co = _csr(list(candidates))
    flat = [r for refs in references for r in refs]
    rt, ro = _csr(flat)
    ri = np.zeros(len(references) + 1, dtype=np.int64)
    if references:
        ri[1:] = np.cumsum([len(r) for r in references])
    out = np.zeros(len(candidates), dtype=np.float64)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    _lib.check(lib.capk_cider_d(len(candidates), p(ct), p(co), p(rt), p(ro), p(ri), int(n), float(sigma),
                                int(threads), p(out)), "capk_cider_d")
    return out
