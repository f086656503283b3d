"""Host-side runtime pieces that need no GPU: the decode-runner cache shared by the SCST
sampler and the baseline-search thread (capk.graphs.runner_for), and the trainer's explicit
sampler epochs (capk.train.trainer._set_epoch)."""
import threading

import pytest  # noqa: F401


class _Dec:
    pass


class _Runner:
    pass


def test_runner_cache_is_thread_safe_under_eviction():
    from capk import graphs
    graphs.clear()
    decs = [_Dec() for _ in range(3)]
    errors = []
    made = []

    def worker(tid):
        try:
            for i in range(3000):
                d = decs[(i + tid) % len(decs)]
                key = (i * 7 + tid) % (graphs.MAX_RUNNERS + 4)  # more keys than the cache holds
                r = graphs.runner_for(d, key, lambda: made.append(1) or _Runner())
                assert r.owner is d
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:3]
    assert len(graphs._RUNNERS) <= graphs.MAX_RUNNERS
    graphs.clear()


def test_runner_cache_drops_entry_of_a_dead_decoder_with_reused_id():
    from capk import graphs
    graphs.clear()
    d1 = _Dec()
    r1 = graphs.runner_for(d1, "k", _Runner)
    assert graphs.runner_for(d1, "k", _Runner) is r1
    # simulate id() reuse: a different object presenting the same cache key
    k = next(iter(graphs._RUNNERS))
    d2 = _Dec()
    graphs._RUNNERS[(id(d2), "k")] = graphs._RUNNERS.pop(k)
    r2 = graphs.runner_for(d2, "k", _Runner)
    assert r2 is not r1 and r2.owner is d2
    graphs.clear()


def test_trainer_sets_sampler_epoch_per_pass():
    from capk.data import EpochSampler
    from capk.train.trainer import _set_epoch

    class L:
        sampler = EpochSampler(10, seed=3)

    _set_epoch(L, 4)
    a = list(iter(L.sampler))
    _set_epoch(L, 4)
    b = list(iter(L.sampler))
    assert a == b and all(ep == 4 for _, ep in a)
    _set_epoch(L, 5)
    assert all(ep == 5 for _, ep in iter(L.sampler))
