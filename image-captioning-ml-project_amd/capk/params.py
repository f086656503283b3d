"""Flat parameter storage for the capk hot path.

Every parameter of a model is re-homed into one of two flat fp32 *master*
buffers — weight-decay and no-weight-decay, following the reference's AdamW
group rule (src/train/trainer.py:114-128) — with a parallel flat fp32 gradient
buffer and a flat bf16 *shadow* used by the bf16 kernels.  ``p.data``,
``p.grad``, ``p._capk_grad`` and ``p._capk_bf16`` are views into those buffers,
so:

* the fused AdamW kernel updates a whole group in one launch and refreshes the
  bf16 shadow in the same pass (no separate cast kernel per step);
* parameters that are consumed together (q/k/v projections) are laid out
  adjacently and exposed as one fused [3D, D] matrix (``Fused``), so the QKV
  projection is a single GEMM;
* data-parallel gradient all-reduce works on large contiguous buckets.

Parameters that the reference leaves without a gradient in some
configurations (the ViT pooler when the decoder ignores ``pooled_features``:
torch AdamW then skips them) are placed at the tail of their buffer and marked
optional; the optimizer only updates them in steps where a backward wrote them.
Frozen parameters (``requires_grad=False``, e.g. ``EncoderConfig.freeze``) sit
behind those and are never handed to the optimizer: the reference builds its
AdamW groups from ``p.requires_grad`` parameters only (trainer.py:117-126).
"""
import torch

ALIGN = 16  # elements: keeps every view 64-B (fp32) / 32-B (bf16) aligned


def no_decay(name):
    """trainer.py:114-128: names containing 'bias' or 'LayerNorm.weight' skip weight decay."""
    return any(nd in name for nd in ("bias", "LayerNorm.weight"))


def _round(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


def _alloc_numel(p):
    lay = getattr(p, "_capk_layout", None)
    if lay is not None:
        n = 1
        for d in lay[0]:
            n *= d
        return n
    pr = getattr(p, "_capk_pad_rows", None)
    if pr:
        assert pr >= p.shape[0]
        return pr * (p.numel() // p.shape[0])
    return p.numel()


class Fused:
    """Adjacent parameters exposed as one matrix: master / bf16 / grad views."""

    def __init__(self, params):
        self.params = list(params)
        self.master = self.bf16 = self.grad = None

    def w(self, dtype):
        return self.bf16 if dtype == torch.bfloat16 else self.master


class ParamStore:
    def __init__(self, model, device, bf16_shadow=True):
        self.device = torch.device(device)
        named = list(model.named_parameters())
        self.named = named  # reference order (torch optimizer state-dict numbering)
        names = {id(p): n for n, p in named}
        fused = []
        for m in model.modules():
            fn = getattr(m, "_capk_fused_groups", None)
            if fn is not None:
                fused.extend(fn())
        in_fused = {}
        for f in fused:
            for p in f.params:
                in_fused[id(p)] = f
        self.groups = {"decay": [], "no_decay": []}
        self.optional = set()
        for m in model.modules():
            for p in getattr(m, "_capk_optional_params", lambda: [])():
                self.optional.add(id(p))
        self.frozen = {id(p) for _, p in named if not p.requires_grad}
        # order: registration order, a fused group placed (adjacent) at its first member;
        # optional-grad parameters last within each buffer.  The backward finishes the
        # modules in reverse registration order, so the final gradients of each buffer
        # grow as a suffix (dp.GradBucketer launches its all-reduce buckets from that).
        seen = set()
        order = []
        for _, p in named:
            for q in (in_fused[id(p)].params if id(p) in in_fused else (p,)):
                if id(q) not in seen:
                    seen.add(id(q))
                    order.append(q)
        # a module whose backward finishes some of its parameters LAST (the decoder's visual
        # projection, after every layer) lists them in _capk_store_first(): they move to the
        # front of the module's run, so its layers' gradients still grow as a suffix
        for m in model.modules():
            fn = getattr(m, "_capk_store_first", None)
            if fn is None:
                continue
            first = [q for q in fn() if q is not None]
            ids = {id(q) for q in first}
            own = {id(q) for q in m.parameters()}
            at = min(i for i, q in enumerate(order) if id(q) in own)
            rest = [q for q in order if id(q) not in ids]
            at = sum(1 for q in order[:at] if id(q) not in ids)
            order = rest[:at] + first + rest[at:]
        for p in order:
            g = "no_decay" if no_decay(names[id(p)]) else "decay"
            self.groups[g].append(p)
        def tail_rank(p):  # stable sort: required, then optional, then frozen
            return 2 if id(p) in self.frozen else int(id(p) in self.optional)

        for g in self.groups:
            self.groups[g].sort(key=tail_rank)
        self.master, self.grad, self.bf16, self.offsets = {}, {}, {}, {}
        self.required_numel = {}
        self.params = []
        self.names = {}
        for g, plist in self.groups.items():
            total = sum(_round(_alloc_numel(p)) for p in plist)
            master = torch.zeros(max(total, ALIGN), dtype=torch.float32, device=self.device)
            grad = torch.zeros_like(master)
            shadow = torch.zeros(master.numel(), dtype=torch.bfloat16, device=self.device) if bf16_shadow else None
            off = 0
            req = 0
            for p in plist:
                n = p.numel()
                lay = getattr(p, "_capk_layout", None)
                if lay is not None:
                    # kernel-native storage (e.g. channels-last, K-padded conv weights):
                    # the parameter is a strided view of its storage block
                    sshape, view = lay
                    ns = _alloc_numel(p)
                    ms = master[off:off + ns].view(sshape)
                    with torch.no_grad():
                        view(ms).copy_(p.detach().to(self.device, torch.float32))
                    p.data = view(ms)
                    p._capk_master_store = ms
                    p._capk_grad_store = grad[off:off + ns].view(sshape)
                    p._capk_grad = view(p._capk_grad_store)
                    p.grad = p._capk_grad
                    if shadow is not None:
                        p._capk_bf16_store = shadow[off:off + ns].view(sshape)
                        p._capk_bf16 = view(p._capk_bf16_store)
                else:
                    with torch.no_grad():
                        master[off:off + n].copy_(p.detach().reshape(-1).to(self.device, torch.float32))
                    p.data = master[off:off + n].view(p.shape)
                    p._capk_grad = grad[off:off + n].view(p.shape)
                    p.grad = p._capk_grad
                    if shadow is not None:
                        p._capk_bf16 = shadow[off:off + n].view(p.shape)
                pr = getattr(p, "_capk_pad_rows", None)
                if pr:
                    # zero-padded row extension (e.g. vocab rounded up for the GEMM tiles)
                    pshape = (pr,) + tuple(p.shape[1:])
                    npad = _alloc_numel(p)
                    p._capk_pad_master = master[off:off + npad].view(pshape)
                    p._capk_pad_grad = grad[off:off + npad].view(pshape)
                    p._capk_pad_bf16 = None if shadow is None else shadow[off:off + npad].view(pshape)
                p._capk_store_ref = self
                p._capk_group = g
                p._capk_offset = off
                self.offsets[id(p)] = (g, off)
                self.names[id(p)] = names[id(p)]
                off += _round(_alloc_numel(p))
                if id(p) not in self.optional and id(p) not in self.frozen:
                    req = off
                self.params.append(p)
            self.master[g], self.grad[g], self.bf16[g] = master, grad, shadow
            if shadow is not None and shadow.is_cuda:
                from . import ops
                ops.WT.register(shadow)
            self.required_numel[g] = req
        for f in fused:
            self._bind_fused(f)
        self.written_optional = set()
        self.refresh_shadow()

    def _bind_fused(self, f):
        g, off0 = self.offsets[id(f.params[0])]
        off = off0
        for p in f.params:
            assert self.offsets[id(p)] == (g, off), "fused parameters must be adjacent in one group"
            off += _round(p.numel())
            assert _round(p.numel()) == p.numel(), "fused parameters must have ALIGN-multiple sizes"
        rows = sum(p.shape[0] for p in f.params)
        shape = (rows,) + tuple(f.params[0].shape[1:])
        n = off - off0
        f.master = self.master[g][off0:off0 + n].view(shape)
        f.grad = self.grad[g][off0:off0 + n].view(shape)
        f.bf16 = None if self.bf16[g] is None else self.bf16[g][off0:off0 + n].view(shape)

    def refresh_shadow(self):
        """Re-derive the bf16 shadow after the master weights changed outside the optimizer."""
        from . import ops
        ops.FP8.weights_changed()
        ops.WT.join()
        ops.WT.weights_changed()
        for g in self.groups:
            if self.bf16[g] is not None and self.master[g].is_cuda:
                ops.cast(self.master[g], self.bf16[g])
            elif self.bf16[g] is not None:
                self.bf16[g].copy_(self.master[g])

    def param_view(self, p, bufs):
        """`p`-shaped view into a flat buffer dict laid out like the master buffers
        (e.g. the optimizer's moments)."""
        g, off = self.offsets[id(p)]
        lay = getattr(p, "_capk_layout", None)
        if lay is not None:
            sshape, view = lay
            return view(bufs[g][off:off + _alloc_numel(p)].view(sshape))
        return bufs[g][off:off + p.numel()].view(p.shape)

    def mark_written(self, p):
        if id(p) in self.optional and id(p) not in self.frozen:
            self.written_optional.add(id(p))

    def relink_grads(self):
        for p in self.params:
            if p.grad is None or p.grad.data_ptr() != p._capk_grad.data_ptr():
                p.grad = p._capk_grad

    def segments(self, group):
        """[(key, start, end)] ranges of `group` to update this step.  Keys are stable so the
        optimizer can keep per-range step counts (torch AdamW keeps a step count per
        parameter; optional parameters advance only in steps that produced a gradient)."""
        segs = [((group, "required"), 0, self.required_numel[group])] if self.required_numel[group] else []
        for p in self.groups[group]:
            if id(p) in self.optional and id(p) in self.written_optional and id(p) not in self.frozen:
                off = p._capk_offset
                segs.append(((group, off), off, off + _round(_alloc_numel(p))))
        return segs


def store_of(module):
    return getattr(module, "_capk_store", None)


def notify_final(store, params=None, all_except=None):
    """Tell the store's gradient bucketer (dp.GradBucketer, if one is installed) that the
    gradients of `params` -- or of every parameter not in `all_except` -- are final for
    this backward.  No-op without a bucketer (single process)."""
    b = getattr(store, "_capk_bucketer", None) if store is not None else None
    if b is None or not b.active:
        return
    if all_except is not None:
        skip = {id(p) for p in all_except}
        ids = [id(p) for p in store.params if id(p) not in skip]
    else:
        ids = [id(p) for p in params]
    b.mark_final(ids)


def attach(model, device, bf16_shadow=True):
    """Build the ParamStore for `model` and remember it on every submodule."""
    st = ParamStore(model, device, bf16_shadow)
    for m in model.modules():
        m._capk_store = st
    return st
