"""Oracle for the SCST sampler.  TEST INFRASTRUCTURE ONLY.

Restates capk's Categorical sampler: the distribution of the reference's
``torch.distributions.Categorical(softmax(logits)).sample()`` (src/train/trainer.py:420-426)
drawn by inverse CDF with the counter-based uniform u = (hash(seed, step<<32 | row) >> 8) / 2^24
(the dropout hash of csrc/common.h), CDF accumulated in fp32 over 256 contiguous
column chunks in order — the same arithmetic order as the kernel, so tokens agree
except when u*S falls within rounding of a CDF boundary (reported by ``margin``).
"""
import numpy as np


def drop_hash(seed, idx):
    m = 0xFFFFFFFF
    x = (seed ^ (((idx & m) * 0x9E3779B9) & m) ^ ((((idx >> 32) & m) * 0x7FEB352D) & m)) & m
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & m
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & m
    x ^= x >> 16
    return x


def uniform(seed, step, row):
    return np.float32((drop_hash(seed & 0xFFFFFFFF, ((step & 0xFFFFFFFF) << 32) | row) >> 8) * (1.0 / 16777216.0))


def sample_row(x, seed, step, row):
    """x: float32 [V] logits -> (token, logp, margin)."""
    x = np.asarray(x, dtype=np.float32)
    V = x.shape[0]
    chunk = (V + 255) // 256
    M = np.float32(x.max())
    e = np.exp((x - M).astype(np.float32)).astype(np.float32)
    part = np.array([np.float32(np.sum(e[t * chunk:min(V, (t + 1) * chunk)], dtype=np.float32)) for t in range(256)],
                    dtype=np.float32)
    S = np.float32(np.sum(part, dtype=np.float32))
    target = np.float32(uniform(seed, step, row) * S)
    cdf = np.cumsum(e.astype(np.float64))
    tok = int(np.searchsorted(cdf, float(target), side="right"))
    tok = min(tok, V - 1)
    margin = float(np.min(np.abs(cdf - float(target)))) / float(S)
    logp = float(x[tok] - M) - float(np.log(np.float64(S)))
    return tok, logp, margin
