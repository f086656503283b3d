"""Data parallelism: one process per GPU, gradient all-reduce over RCCL/xGMI.

The reference has no distributed code; the build adds plain DP
(SURVEY §8e): every rank computes the full train step on its own batch shard and
the flat fp32 gradient buffers of the ParamStore are averaged with bucketed
``all_reduce`` (backend "nccl" = RCCL on ROCm).  Buckets are contiguous slices
of the flat buffers (no packing copies).

``GradBucketer`` overlaps that exchange with the backward.  Model code reports
when gradients are final (``params.notify_final``: the Transformer / GPT-2 decoder's LM
head and each of its layers as the backward leaves them, each encoder layer at the end
of its backward, the encoder head once the decoder and the head are done).  The
flat buffers are laid out in registration order (params.py) and the backward
finishes the modules in reverse order, so in every buffer the final gradients
form a growing suffix.  Whenever that suffix has grown by a bucket, the bucketer
launches ``all_reduce(async_op=True)`` on it: RCCL runs the collective on its own
stream, ordered after the work already queued on the compute stream, while the
compute stream carries on with the next layer's backward.  ``finish()`` launches
the remainder and makes the compute stream wait for every collective before the
optimizer step.  Every rank issues the same collectives in the same order (the
notifications follow the same backward on every rank).

``exchange="bf16"`` halves the wire bytes (SURVEY §5 budgets bf16): each bucket is cast
to a bf16 staging copy on the compute stream, the all-reduce runs on the copy, and
``finish()`` writes the averaged values back into the fp32 gradient buffer (the fp32
master weights and moments are untouched; only the exchanged gradient is rounded to
bf16, once per rank and once per ring reduction step).
"""
import torch
import torch.distributed as dist

from ..params import _alloc_numel, _round

BUCKET_ELEMS = 16 * 1024 * 1024  # 64 MiB of fp32 per all-reduce


def _active():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _avg_op():
    if dist.get_backend() == "nccl":
        return dist.ReduceOp.AVG, False
    return dist.ReduceOp.SUM, True  # gloo has no AVG: sum, then scale


def allreduce_grads(store, bucket_elems=BUCKET_ELEMS):
    """Average every gradient buffer across ranks (blocking on the current stream)."""
    if not _active():
        return
    op, need_scale = _avg_op()
    world = dist.get_world_size()
    for g in store.groups:
        buf = store.grad[g]
        n = buf.numel()
        for s in range(0, n, bucket_elems):
            chunk = buf[s:s + bucket_elems]
            dist.all_reduce(chunk, op=op)
            if need_scale:
                chunk.div_(world)


class GradBucketer:
    """Backward-overlapped gradient averaging for one ParamStore.

    Per step: ``loss.backward(); bucketer.finish(); optimizer.step()``.
    Installs itself on the store (``store._capk_bucketer``) so model code can notify it.
    """

    def __init__(self, store, bucket_elems=BUCKET_ELEMS, exchange="fp32"):
        if exchange not in ("fp32", "bf16"):
            raise ValueError(f"GradBucketer: exchange must be 'fp32' or 'bf16', got {exchange!r}")
        self.store = store
        self.bucket_elems = int(bucket_elems)
        self.exchange = exchange
        self.active = _active()
        # bf16 staging buffers, one per gradient group, laid out like the fp32 buffers
        self.stage = ({g: torch.empty(b.numel(), dtype=torch.bfloat16, device=b.device) for g, b in store.grad.items()}
                      if exchange == "bf16" and self.active else None)
        # per group: [start, end) of every parameter, in buffer order
        self.spans = {}
        # the buffer tail the store keeps for optional-gradient parameters (e.g. the ViT pooler
        # when the decoder ignores pooled_features) and frozen ones: not part of the growing
        # suffix -- an optional parameter is written (if at all) by the encoder head, late in the
        # backward, and would hold back every decoder bucket in front of it -- but exchanged by
        # finish() once the whole backward is done ([tail0, opt_end): the optional ones)
        self.tail0, self.opt_end, self.ntail = {}, {}, {}
        late = set(store.frozen) | set(store.optional)
        for g, plist in store.groups.items():
            self.spans[g] = sorted((p._capk_offset, p._capk_offset + _round(_alloc_numel(p)), id(p)) for p in plist)
            tail = [sp for sp in self.spans[g] if sp[2] in late]
            self.ntail[g] = len(tail)
            n = store.grad[g].numel()
            self.tail0[g] = tail[0][0] if tail else n
            frozen = [sp for sp in self.spans[g] if sp[2] in store.frozen]
            self.opt_end[g] = frozen[0][0] if frozen else n
            assert all(sp[2] in late for sp in self.spans[g][len(self.spans[g]) - len(tail):]), \
                "GradBucketer: optional / frozen parameters must sit at the buffer tail"
        if self.active:
            self.op, self.need_scale = _avg_op()
            self.world = dist.get_world_size()
        store._capk_bucketer = self
        self.reset()

    def reset(self):
        # frozen parameters never receive a gradient; optional ones are exchanged by finish()
        self.final = set(self.store.frozen) | set(self.store.optional)
        self.works = []
        self.k = dict(self.ntail)                                  # spans known final, counted from the end
        self.lo = dict(self.tail0)                                 # start of the final suffix
        self.hi = dict(self.lo)                                    # [hi, tail0) already launched

    def mark_final(self, ids):
        self.final.update(ids)
        for g, spans in self.spans.items():
            n = len(spans)
            while self.k[g] < n and spans[n - 1 - self.k[g]][2] in self.final:
                self.lo[g] = spans[n - 1 - self.k[g]][0]
                self.k[g] += 1
            if self.hi[g] - self.lo[g] >= self.bucket_elems:
                self._launch(g, self.lo[g], self.hi[g])
                self.hi[g] = self.lo[g]

    def _launch(self, g, lo, hi):
        buf = self.store.grad[g]
        for s in range(lo, hi, self.bucket_elems):
            chunk = buf[s:min(hi, s + self.bucket_elems)]
            if self.stage is not None:
                wire = self.stage[g][s:min(hi, s + self.bucket_elems)]
                _cast(chunk, wire)
            else:
                wire = chunk
            self.works.append((dist.all_reduce(wire, op=self.op, async_op=True), chunk, wire))

    def finish(self):
        """Launch what is left, then join every collective (the current stream waits)."""
        if self.active:
            for g in self.spans:
                if self.hi[g] > 0:
                    self._launch(g, 0, self.hi[g])
                if self.opt_end[g] > self.tail0[g]:  # the optional tail, final now
                    self._launch(g, self.tail0[g], self.opt_end[g])
            for work, chunk, wire in self.works:
                work.wait()
                if wire is not chunk:
                    _cast(wire, chunk)
                if self.need_scale:
                    chunk.div_(self.world)
        self.reset()


def _cast(src, dst):
    """dst <- src (fp32 <-> bf16) on the current stream: the capk cast kernel on the GPU,
    torch on the CPU (gloo tests)."""
    if src.is_cuda:
        from .. import ops
        ops.cast(src, dst)
    else:
        dst.copy_(src)
