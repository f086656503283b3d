"""Host-side bookkeeping of ops.WeightT (the K-major weight copies for the dX products):
ownership by live ParamStore shadows, invalidation on new stores / weight changes, and the
cases that must keep the N-major operand.  No kernels run (CPU tensors)."""
import gc

import torch

from capk import ops


def _fresh():
    wt = ops.WeightT()
    wt.enabled = True
    return wt


def test_ownership_follows_live_shadows():
    wt = _fresh()
    buf = torch.zeros(4096, dtype=torch.bfloat16)
    e0 = wt.epoch
    wt.register(buf)
    assert wt.epoch == e0 + 1  # a new store: every copy is stale
    w = buf[:2048].view(32, 64)
    assert wt._owned(w)
    assert wt._owned(buf[1024:3072].view(64, 32))
    assert not wt._owned(torch.zeros(32, 64, dtype=torch.bfloat16))  # outside any shadow
    assert not wt._owned(buf.new_zeros(5000)[:2048].view(32, 64))
    # a freed store's range stops counting, and its cache entries are pruned on the next register
    wt.cache[(torch.device("cpu"), w.data_ptr(), 32, 64, 64)] = [wt.epoch, None]
    del w
    del buf
    gc.collect()
    other = torch.zeros(16, dtype=torch.bfloat16)
    wt.register(other)
    assert len(wt.buffers) == 1 and not wt.cache


def test_get_declines_unsupported_products():
    wt = _fresh()
    buf = torch.zeros(4096, dtype=torch.bfloat16)
    wt.register(buf)
    w = buf[:2048].view(32, 64)
    assert wt.get(w, 4096) is None  # CPU tensor: no device copy
    wt.enabled = False
    assert wt.get(w, 4096) is None
    wt.enabled = True
    assert wt.get(w.float(), 4096) is None  # fp32 weights
    assert wt.get(w, 16) is None  # short products keep the N-major weight
    wt.weights_changed()
    e = wt.epoch
    wt.weights_changed()
    assert wt.epoch == e + 1


def test_refresh_async_and_join_are_noops_without_gpu_work():
    wt = _fresh()
    wt.overlap = True
    wt.refresh_async()  # nothing cached: nothing launched
    wt.join()
    assert not wt.pending
