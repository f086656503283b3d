"""Tensor-level wrappers over the C ABI (device pointers + current HIP stream).

Every function here launches hand-written HIP kernels from libcapk.so on
``torch.cuda.current_stream()``; torch is used only for memory (caching
allocator), streams and autograd bookkeeping.  There is deliberately no CPU or
eager-PyTorch fallback: a missing library or a non-GPU tensor raises.
"""

import ctypes
import contextlib
import os
import threading
import weakref

import torch

from . import _lib
from ._lib import ACT_BWD, BF16, F32, check  # noqa: F401

_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dtype_code(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise _lib.CapkError(f"capk: unsupported dtype {t.dtype}")


def _p(t):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _need_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.CapkError("capk ops need device (HIP) tensors; there is no CPU path")


def _ws(nbytes, device):
    if nbytes == 0:
        return None
    return torch.empty(int(nbytes), dtype=torch.uint8, device=device)


def lib():
    return _lib.load()


# ------------------------------------------------------ deferred finishes ---
# capk_finish_defer (include/capk.h): inside `deferred_finishes()` the column-sum / LayerNorm
# partial-sum finishes are queued per stream and launched as one kernel per stream at exit
# (the same sums, bit-identical); the workspaces they read are held here until then.
# CAPK_FINISH_DEFER=0: every finish launches at once (A/B).
_FIN = threading.local()
_FIN_ON = os.environ.get("CAPK_FINISH_DEFER", "1") != "0"


def _hold(ws):
    """Keep a workspace whose finish may be queued alive until the context's flush."""
    h = getattr(_FIN, "hold", None)
    if h is not None and ws is not None:
        h.append(ws)


@contextlib.contextmanager
def deferred_finishes():
    """One launch for the partial-sum finishes issued inside (a layer's backward)."""
    if not _FIN_ON or getattr(_FIN, "hold", None) is not None:  # off, or nested: the outer one flushes
        yield
        return
    L = lib()
    _FIN.hold = []
    check(L.capk_finish_defer(1), "capk_finish_defer")
    try:
        yield
    finally:
        try:
            check(L.capk_finish_flush_all(), "capk_finish_flush_all")
        finally:
            L.capk_finish_defer(0)
            # the flushes are enqueued: a later kernel reusing these blocks runs after them
            _FIN.hold = None


# ------------------------------------------------------------------- GEMM ---
class KernelTimer:
    """Optional HIP-event bracketing of every GEMM launch on the current stream
    (bench.py's live roofline measurement).  Off by default: zero overhead."""

    def __init__(self):
        self.enabled = False
        self.stream = None
        self.records = []  # (start_event, end_event, flops, in_dtype, algorithmic HBM bytes)
        # every `stride`-th launch is bracketed: an event pair costs ~3 us of GPU time (config 3:
        # events on all 279 launches of a step cost 3.7 % of the step); the per-step launch
        # sequence (279 launches) is coprime to the default stride, so successive steps sample
        # every launch position
        self.stride = max(1, int(os.environ.get("CAPK_GEMM_TIMER_STRIDE", "5")))
        self.seen = 0

    def start(self):
        """Record the GEMMs launched on the calling thread's current stream, from any thread:
        the backward runs on autograd's device thread with the forward's stream current, while
        the config-5 SCST baseline search runs on its own side stream from a second host thread
        (its overlapping, mutually stretched launches would otherwise be summed in) -- as do the
        weight gradients under CAPK_DW_STREAM=1."""
        self.records = []
        self.seen = 0
        self.stream = torch.cuda.current_stream().cuda_stream
        self.enabled = True

    def active(self):
        if not (self.enabled and not torch.cuda.is_current_stream_capturing()
                and torch.cuda.current_stream().cuda_stream == self.stream):
            return False
        self.seen += 1
        return (self.seen - 1) % self.stride == 0

    def stop(self):
        self.enabled = False

    def summary(self):
        torch.cuda.synchronize()
        tot_ms, tot_flops, tot_bytes, n = 0.0, 0.0, 0.0, 0
        route = {0: [0, 0.0, 0.0], 2: [0, 0.0, 0.0]}  # per path (0: bf16 kernels, 2: fp8): launches, ms, flops
        for s, e, fl, _, by, rt in self.records:
            ms = s.elapsed_time(e)
            tot_ms += ms
            tot_flops += fl
            tot_bytes += by
            n += 1
            route[rt][0] += 1
            route[rt][1] += ms
            route[rt][2] += fl
        by_route = {name: {"launches": r[0], "total_ms": r[1], "tflops": (r[2] / (r[1] * 1e-3) / 1e12) if r[1] else 0.0}
                    for name, r in (("gemm_bf16_kernel", route[0]), ("gemm_f8", route[2]))}
        return {"launches": n, "total_ms": tot_ms, "flops": tot_flops, "by_route": by_route,
                "avg_ms": tot_ms / max(n, 1), "avg_flops": tot_flops / max(n, 1), "avg_bytes": tot_bytes / max(n, 1),
                "stride": self.stride, "launches_seen": self.seen}


GEMM_TIMER = KernelTimer()


NO_DROP = (0.0, 0)


def gemm(A, a_kmajor, B, b_kmajor, M, N, K, C, *, lda, ldb, ldc, alpha=1.0, beta=0.0, bias=None,
         residual=None, ldr=0, act=0, preact=None, aux=None, ldx=0, drop=NO_DROP):
    """C[m,n] = alpha*sum_k A(m,k)B(n,k) + beta*C + bias + residual -> act (see capk.h)."""
    _need_gpu(A, B, C)
    L = lib()
    it, ot = dtype_code(A), dtype_code(C)
    wsb = L.capk_gemm_workspace(it, ot, M, N, K)
    ws = _ws(wsb, A.device)
    timed = GEMM_TIMER.active()
    if timed:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    rc = L.capk_gemm(it, ot, M, N, K, _p(A), lda, int(a_kmajor), _p(B), ldb, int(b_kmajor), _p(C), ldc,
                     float(alpha), float(beta), _p(bias), _p(residual), ldr, int(act), _p(preact), _p(aux), ldx,
                     float(drop[0]), int(drop[1]) & 0xFFFFFFFF, _p(ws), wsb if ws is not None else 0, _stream())
    check(rc, "capk_gemm")
    if timed:
        ev1.record()
        # algorithmic bytes: A and B read once, C written once (+ read when beta != 0), and each
        # side stream once (residual / aux read, pre-activation written)
        ein, eout = A.element_size(), C.element_size()
        sides = (1 if beta else 0) + (residual is not None) + (aux is not None) + (preact is not None)
        nbytes = ein * (M * K + N * K) + eout * M * N * (1 + sides)
        GEMM_TIMER.records.append((ev0, ev1, 2.0 * M * N * K, it, nbytes, 0))
    return C


# ------------------------------------------------------------------- fp8 ----
class Fp8State:
    """Config 5's fp8 forward (BASELINE configs[4]): when enabled (capk.prepare(...,
    precision='fp8')), forward Linear / Conv1D products whose weight lives in the model's
    ParamStore and whose grid fills the chip run as e4m3 x e4m3 scaled-MFMA GEMMs
    (capk_gemm_f8); the activation is quantised per row on the fly, the weight once per
    optimizer step (lazily, on first use after `weights_changed`).  Backward products stay
    bf16 against the bf16 weights and the saved bf16 activations."""

    def __init__(self):
        self.enabled = False
        self.epoch = 0
        self.ranges = []  # (start, end) byte ranges of the ParamStore bf16 shadows
        self.cache = {}   # (ptr, shape, stride, transposed) -> [epoch, q, scale]
        self.min_rows = 256  # products with fewer rows (decode steps of small batches) stay bf16
        self.min_ctas = 96  # 256x256 tiles (x2 for K >= 2048) below which the bf16 kernels run instead

    def enable(self, store):
        self.ranges = [(b.data_ptr(), b.data_ptr() + b.numel() * b.element_size())
                       for b in store.bf16.values() if b is not None]
        self.cache.clear()
        self.enabled = True

    def disable(self):
        self.enabled = False
        self.cache.clear()

    def weights_changed(self):
        self.epoch += 1

    def refresh(self):
        """Re-quantise every cached weight copy that is stale (before a graph replay: a
        captured graph holds the copies' addresses, never the quantisation itself)."""
        if not self.enabled:
            return
        for key, ent in list(self.cache.items()):  # snapshot: another thread may insert; ent = [epoch, q, scale, view]
            if ent[0] != self.epoch:
                quant_fp8(ent[3], transpose=key[3], q=ent[1], scale=ent[2])
                ent[0] = self.epoch

    def is_weight(self, w):
        p = w.data_ptr()
        return any(a <= p < b for a, b in self.ranges)


FP8 = Fp8State()


class _TransposeDesc(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("ld_src", ctypes.c_int64),
                ("ld_dst", ctypes.c_int64), ("rows", ctypes.c_int32), ("cols", ctypes.c_int32)]


class WeightT:
    """K-major copies of the bf16 weights for the backward's dX products.

    dX = dY W reads W [N_out][K_in] N-major; the same product with W^T [K_in][N_out] runs on the
    K-major GEMM paths, 3-30 % faster on the config-3 shapes (profiles/round6/dx_kmajor.txt:
    e.g. the ViT QKV dX 206 -> 182 us, the decoder FC1 dX 51 -> 36 us).  A copy is made the
    first time a ParamStore weight reaches `linear_dx` and refreshed once per optimizer step
    (`weights_changed`): the first dX product after a change re-transposes every known copy on
    that device in one batched launch (capk_transpose_bf16_batch).  Views outside a live
    ParamStore bf16 shadow, fp32 weights, products under graph capture and short products
    (M < 2048 rows) keep the N-major operand.  CAPK_WT=0 turns the copies off (A/B)."""

    MIN_ROWS = 2048
    MAX_DIM = 8192  # (the LM-head dX, K = 50 304, stays on its split-K path)

    def __init__(self):
        self.enabled = os.environ.get("CAPK_WT", "1") != "0"
        # (opt-in: measured 0.8 % slower on config 3 -- the transposes' 23 k workgroups take the
        # CUs from the forward's first GEMMs; profiles/round6/weight_copies_ab.txt)
        self.overlap = os.environ.get("CAPK_WT_OVERLAP", "0") == "1"
        self.epoch = 0
        self.buffers = []  # (weakref of a ParamStore bf16 shadow, start, end)
        self.cache = {}    # (device, ptr, rows, cols, ld) -> [epoch, W^T]
        self.lock = threading.Lock()
        self.side = {}     # device -> side stream of refresh_async
        self.pending = {}  # device -> event recorded after its refresh on the side stream

    def refresh_async(self):
        """Right after an optimizer step: re-transpose every known copy now, on a side stream
        that waits for the update, so the transposes overlap the next forward; the first dX
        product (get) and the next shadow write (join, from adamw / refresh_shadow) wait for
        them.  Opt-in (CAPK_WT_OVERLAP=1); by default the copies are refreshed by that first dX
        product."""
        if not (self.enabled and self.overlap) or not torch.cuda.is_available() or \
                torch.cuda.is_current_stream_capturing():
            return
        with self.lock:
            for dev in {k[0] for k, e in self.cache.items() if e[0] != self.epoch}:
                side = self.side.get(dev)
                if side is None:
                    side = self.side[dev] = torch.cuda.Stream(device=dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    self._refresh(dev)
                for k, e in self.cache.items():
                    if k[0] == dev:
                        e[1].record_stream(side)
                ev = torch.cuda.Event()
                ev.record(side)
                self.pending[dev] = ev

    def join(self, dev=None):
        """Make the current stream wait for refreshes still running on the side stream."""
        if not self.pending:
            return
        with self.lock:
            for d in [d for d in self.pending if dev is None or d == dev]:
                torch.cuda.current_stream(d).wait_event(self.pending.pop(d))

    def register(self, buf):
        """A new ParamStore shadow: its memory may be a freed store's, so every copy goes stale."""
        with self.lock:
            self._prune()
            self.buffers.append((weakref.ref(buf), buf.data_ptr(), buf.data_ptr() + buf.numel() * buf.element_size()))
            self.epoch += 1

    def weights_changed(self):
        self.epoch += 1

    def _prune(self):
        dead = [(a, b) for r, a, b in self.buffers if r() is None]
        if dead:
            self.buffers = [e for e in self.buffers if e[0]() is not None]
            self.cache = {k: v for k, v in self.cache.items() if not any(a <= k[1] < b for a, b in dead)}

    def _owned(self, w):
        p = w.data_ptr()
        end = p + ((w.shape[0] - 1) * w.stride(0) + w.shape[1]) * w.element_size()
        return any(r() is not None and a <= p and end <= b for r, a, b in self.buffers)

    def get(self, w, M):
        """W^T for the dX product of M rows against `w`, or None (use `w` N-major)."""
        if not self.enabled or M < self.MIN_ROWS or w.dtype != torch.bfloat16 or not w.is_cuda or w.dim() != 2:
            return None
        rows, cols = w.shape
        if (w.stride(1) != 1 or rows % 8 or cols % 8 or w.stride(0) % 8 or w.data_ptr() % 16
                or max(rows, cols) > self.MAX_DIM or torch.cuda.is_current_stream_capturing()):
            return None
        with self.lock:
            if not self._owned(w):
                return None
            key = (w.device, w.data_ptr(), rows, cols, w.stride(0))
            ent = self.cache.get(key)
            if ent is None:
                ent = self.cache[key] = [None, torch.empty(cols, rows, dtype=torch.bfloat16, device=w.device)]
            if ent[0] != self.epoch:
                self._refresh(w.device)
            ev = self.pending.pop(w.device, None)
            if ev is not None:  # (refresh_async)
                torch.cuda.current_stream(w.device).wait_event(ev)
            return ent[1]

    def _refresh(self, dev):
        stale = [(k, e) for k, e in self.cache.items() if k[0] == dev and e[0] != self.epoch]
        _transpose_batch([(k[1], k[4], k[2], k[3], e[1]) for k, e in stale])
        for _, e in stale:
            e[0] = self.epoch


def _transpose_batch(items):
    """[(src pointer, src row stride, rows, cols, dst [cols, rows] bf16 tensor)] -> one
    capk_transpose_bf16_batch call (one launch per 64 matrices)."""
    descs = (_TransposeDesc * max(1, len(items)))()
    for i, (src, ld, rows, cols, dst) in enumerate(items):
        descs[i] = _TransposeDesc(src, dst.data_ptr(), ld, dst.stride(0), rows, cols)
    check(lib().capk_transpose_bf16_batch(len(items), ctypes.cast(descs, ctypes.c_void_p), _stream()),
          "capk_transpose_bf16_batch")


def transpose_bf16_batch(pairs):
    """dst <- src^T for every (src [R, C], dst [C, R]) bf16 pair (unit column strides), in one
    batched launch per 64 pairs."""
    for src, dst in pairs:
        _need_gpu(src, dst)
        if src.dtype != torch.bfloat16 or dst.dtype != torch.bfloat16 or src.dim() != 2 or \
                src.stride(1) != 1 or dst.stride(1) != 1 or tuple(dst.shape) != (src.shape[1], src.shape[0]):
            raise _lib.CapkError("transpose_bf16_batch: need bf16 src [R, C] and dst [C, R] with unit column strides")
    _transpose_batch([(s.data_ptr(), s.stride(0), s.shape[0], s.shape[1], d) for s, d in pairs])


WT = WeightT()


def quant_fp8(x, *, transpose=False, q=None, scale=None):
    """e4m3fn rows with E8M0 per-row scales (capk_quant_fp8).  transpose: x [K, N] -> q [N, K]."""
    _need_gpu(x)
    rows, cols = (x.shape[1], x.shape[0]) if transpose else x.shape
    if q is None:
        q = torch.empty(rows, cols, dtype=torch.uint8, device=x.device)
    if scale is None:
        scale = torch.empty(rows, dtype=torch.uint8, device=x.device)
    L = lib()
    wsb = L.capk_quant_fp8_workspace(rows, cols, int(transpose))
    ws = _ws(wsb, x.device)
    check(L.capk_quant_fp8(dtype_code(x), rows, cols, _p(x), x.stride(0), int(transpose), _p(q), q.stride(0),
                           _p(scale), _p(ws), wsb, _stream()), "capk_quant_fp8")
    return q, scale


def gemm_f8(a, sa, b, sb, C, *, beta=0.0, bias=None, residual=None, act=0, preact=None, drop=NO_DROP):
    """C = epilogue((2^sa A8) (2^sb B8)^T): A8 [M,K], B8 [N,K] e4m3fn (uint8 storage)."""
    _need_gpu(a, b, C)
    L = lib()
    M, K = a.shape
    N = b.shape[0]
    wsb = L.capk_gemm_f8_workspace(M, N, K)
    ws = _ws(wsb, a.device)
    timed = GEMM_TIMER.active()
    if timed:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    rc = L.capk_gemm_f8(dtype_code(C), M, N, K, _p(a), a.stride(0), _p(sa), _p(b), b.stride(0), _p(sb), _p(C),
                        C.stride(0), float(beta), _p(bias), _p(residual),
                        residual.stride(0) if residual is not None else 0, int(act), _p(preact),
                        preact.stride(0) if preact is not None else 0, float(drop[0]), int(drop[1]) & 0xFFFFFFFF,
                        _p(ws), wsb if ws is not None else 0, _stream())
    check(rc, "capk_gemm_f8")
    if timed:
        ev1.record()
        nbytes = M * K + N * K + M + N + C.element_size() * M * N * (2 if beta else 1)
        GEMM_TIMER.records.append((ev0, ev1, 2.0 * M * N * K, 2, nbytes, 2))
    return C


def _fp8_route(x, w, M, N, K, act, transposed):
    """(q_w, s_w) when this forward product runs in fp8, else None."""
    if not FP8.enabled or x.dtype != torch.bfloat16 or (act & ACT_BWD) or K % 128 or N % 8 or M < FP8.min_rows:
        return None
    if not FP8.is_weight(w):
        return None
    ctas = ((M + 255) // 256) * ((N + 255) // 256)
    if ctas < FP8.min_ctas and not (K >= 2048 and ctas * 2 >= FP8.min_ctas):
        return None
    key = (w.data_ptr(), tuple(w.shape), tuple(w.stride()), transposed)
    ent = FP8.cache.get(key)
    if ent is None:
        if torch.cuda.is_current_stream_capturing():
            raise _lib.CapkError("capk fp8: weight copy created inside a graph capture (warm the path eagerly first)")
        ent = FP8.cache[key] = [-1, torch.empty(N, K, dtype=torch.uint8, device=w.device),
                                torch.empty(N, dtype=torch.uint8, device=w.device), w]
    if ent[0] != FP8.epoch:
        if torch.cuda.is_current_stream_capturing():
            raise _lib.CapkError("capk fp8: stale weight copy inside a graph capture (call FP8.refresh() first)")
        quant_fp8(w, transpose=transposed, q=ent[1], scale=ent[2])
        ent[0] = FP8.epoch
    return ent[1], ent[2]


def _linear_f8(x, qw, sw, out, b, residual, act, preact, drop):
    qx, sx = quant_fp8(x)
    return gemm_f8(qx, sx, qw, sw, out, bias=b, residual=residual, act=act, preact=preact, drop=drop)


def linear(x, w, b=None, *, out=None, residual=None, act=0, preact=None, out_dtype=None, drop=NO_DROP):
    """y = dropout(act(x @ w^T + b)) + residual; x [M,K] (row stride may exceed K), w [N,K] contiguous."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype or x.dtype, device=x.device)
    f8 = _fp8_route(x, w, M, N, K, act, False)
    if f8 is not None:
        return _linear_f8(x, f8[0], f8[1], out, b, residual, act, preact, drop)
    gemm(x, True, w, True, M, N, K, out, lda=x.stride(0), ldb=w.stride(0), ldc=out.stride(0), bias=b,
         residual=residual, ldr=residual.stride(0) if residual is not None else 0, act=act, preact=preact,
         ldx=preact.stride(0) if preact is not None else 0, drop=drop)
    return out


def linear_lse(x, w, b, V):
    """The LM head with the shifted CE's softmax partials (capk_linear_lse): returns
    (y = x w^T + b [M, N], part) where part (fp32, [4 cdiv(N, 256)][M] (max, sum) pairs) is None
    when the product did not run on the persistent kernel (then use shifted_ce as usual)."""
    M, K = x.shape
    N = w.shape[0]
    out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    if (x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or not w.is_contiguous()
            or _fp8_route(x, w, M, N, K, 0, False) is not None):
        return linear(x, w, b, out=out), None
    _need_gpu(x, w, out)
    L = lib()
    pb = L.capk_linear_lse_part_bytes(M, N)
    part = torch.empty(pb // 4, dtype=torch.float32, device=x.device)
    wsb = L.capk_gemm_workspace(BF16, BF16, M, N, K)
    ws = _ws(wsb, x.device)
    done = ctypes.c_int(0)
    timed = GEMM_TIMER.active()
    if timed:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    check(L.capk_linear_lse(M, N, K, _p(x), x.stride(0), _p(w), w.stride(0), _p(b), _p(out), out.stride(0), int(V),
                            _p(part), pb, ctypes.byref(done), _p(ws), wsb if ws is not None else 0, _stream()),
          "capk_linear_lse")
    if timed:  # (algorithmic bytes: x, w read once, C written once, the partials written once)
        ev1.record()
        GEMM_TIMER.records.append((ev0, ev1, 2.0 * M * N * K, BF16, 2 * (M * K + N * K + M * N) + pb, 0))
    return out, (part if done.value else None)


def ce_lse_fwd(logits2d, targets, B, T, V, ignore_index, part):
    """(loss fp32 [2] = (mean, count), lse fp32 [B*T]) of the shifted CE from linear_lse's partials."""
    L = lib()
    M = B * T
    loss = torch.empty(2, dtype=torch.float32, device=logits2d.device)
    lse = torch.empty(M, dtype=torch.float32, device=logits2d.device)
    wsb = (4 + M) * 4  # the forward's share of capk_ce_lse_workspace: the count and the row losses
    ws = _ws(wsb, logits2d.device)
    nparts = part.numel() // (2 * M)
    check(L.capk_ce_lse_fwd(B, T, V, logits2d.stride(0), _p(logits2d), _p(targets), int(ignore_index), _p(part),
                            nparts, _p(lse), _p(loss), _p(ws), wsb, _stream()), "capk_ce_lse_fwd")
    return loss, lse


def ce_lse_bwd(logits2d, targets, B, T, V, ignore_index, lse, loss, grad_scale, dlogits, dbias=None):
    """dlogits (+ the column sums into dbias, written) of the shifted CE from the saved lse / count."""
    L = lib()
    wsb = L.capk_ce_lse_workspace(B, T, logits2d.stride(0))
    ws = _ws(wsb, logits2d.device)
    check(L.capk_ce_lse_bwd(dtype_code(logits2d), B, T, V, logits2d.stride(0), _p(logits2d), _p(targets),
                            int(ignore_index), _p(lse), loss[1:].data_ptr(), _p(grad_scale), _p(dlogits), _p(dbias),
                            _p(ws), wsb, _stream()), "capk_ce_lse_bwd")
    _hold(ws)
    return dlogits


def linear_dx(dy, w, *, out=None, act_bwd=0, aux=None, beta=0.0, drop=NO_DROP, dsum=None):
    """dX[M,K] = dY[M,N] @ W[N,K]  (optionally * act'(aux) * dropout-mask: fused activation backward).
    dsum (fp32 [K], with act_bwd): also the column sums of the result (the bias gradient of the
    Linear that produced aux), fused into the activation pass."""
    M, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(M, K, dtype=dy.dtype, device=dy.device)
    if dsum is not None and act_bwd and beta == 0.0 and drop[0] <= 0:
        if dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and out.dtype == torch.bfloat16:
            # one call: the product x act'(aux) with the column sums (capk_gemm_dx_act_colsum)
            _need_gpu(dy, w, out, aux, dsum)
            L = lib()
            wsb = L.capk_gemm_dx_act_colsum_workspace(M, K, N)
            ws = _ws(wsb, dy.device)
            timed = GEMM_TIMER.active()
            if timed:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                ev0.record()
            wt = WT.get(w, M)
            fn, wop = (L.capk_gemm_dx_act_colsum_wt, wt) if wt is not None else (L.capk_gemm_dx_act_colsum, w)
            check(fn(M, K, N, _p(dy), dy.stride(0), _p(wop), wop.stride(0), _p(out), out.stride(0),
                     int(act_bwd), _p(aux), aux.stride(0), _p(dsum), 0, _p(ws), wsb, _stream()),
                  "capk_gemm_dx_act_colsum")
            _hold(ws)
            if timed:  # A, B, aux read once; C written once
                ev1.record()
                GEMM_TIMER.records.append((ev0, ev1, 2.0 * M * K * N, dtype_code(dy), 2 * (M * N + N * K + 2 * M * K), 0))
            return out
        gemm(dy, True, w, False, M, K, N, out, lda=dy.stride(0), ldb=w.stride(0), ldc=out.stride(0))
        return act_bwd_colsum(out, aux, act_bwd, dsum)
    wt = WT.get(w, M)
    if wt is not None:  # the K-major copy (WeightT)
        w, bk = wt, True
    else:
        bk = False
    gemm(dy, True, w, bk, M, K, N, out, lda=dy.stride(0), ldb=w.stride(0), ldc=out.stride(0), beta=beta,
         act=(ACT_BWD | act_bwd) if act_bwd else 0, aux=aux, ldx=aux.stride(0) if aux is not None else 0,
         drop=drop)
    return out


def linear_dw(dy, x, dw, *, accumulate=False):
    """dW[N,K] (fp32) (+)= dY[M,N]^T @ X[M,K]."""
    M, N = dy.shape
    K = x.shape[1]
    gemm(dy, False, x, False, N, K, M, dw, lda=dy.stride(0), ldb=x.stride(0), ldc=dw.stride(0),
         beta=1.0 if accumulate else 0.0)
    return dw


def colsum(dy, out, accumulate=False):
    """out[n] (+)= sum_m dy[m, n] (bias gradient, fp32)."""
    _need_gpu(dy, out)
    L = lib()
    M, N = dy.shape
    wsb = L.capk_colsum_workspace(M, N)
    ws = _ws(wsb, dy.device)
    check(L.capk_colsum(dtype_code(dy), M, N, _p(dy), dy.stride(0), _p(out), int(accumulate), _p(ws), wsb,
                        _stream()), "capk_colsum")
    _hold(ws)
    return out


def act_bwd_colsum(c, aux, act, db, accumulate=False):
    """c <- c * act'(aux) in place; db (+)= column sums of the result (capk_act_bwd_colsum)."""
    _need_gpu(c, aux, db)
    L = lib()
    M, N = c.shape
    wsb = L.capk_colsum_workspace(M, N)
    ws = _ws(wsb, c.device)
    check(L.capk_act_bwd_colsum(dtype_code(c), M, N, _p(c), c.stride(0), _p(aux), aux.stride(0), int(act), _p(db),
                                int(accumulate), _p(ws), wsb, _stream()), "capk_act_bwd_colsum")
    _hold(ws)
    return c


# -------------------------------------------------------------- LayerNorm ---
def layernorm_fwd(x, w, b, eps, out=None):
    _need_gpu(x)
    rows, cols = x.shape
    if out is None:
        out = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    check(lib().capk_layernorm_fwd(dtype_code(x), rows, cols, _p(x), x.stride(0), _p(w), _p(b), float(eps),
                                   _p(out), out.stride(0), _p(mean), _p(rstd), _stream()), "capk_layernorm_fwd")
    return out, mean, rstd


def layernorm_bwd(dy, x, w, mean, rstd, dw, db, *, dres=None, out=None, accumulate=False, drop=NO_DROP,
                  out_drop=None, dsum=None):
    """dx = LN'(dy) (+ dres); with drop != off also fills out_drop = LN'(dy) * mask;
    dsum (fp32 [cols], optional) (+)= column sums of dx (a fused bias gradient)."""
    L = lib()
    rows, cols = x.shape
    if out is None:
        out = torch.empty_like(x)
    wsb = L.capk_layernorm_bwd_workspace(rows, cols)
    ws = _ws(wsb, x.device)
    check(L.capk_layernorm_bwd(dtype_code(x), rows, cols, _p(dy), dy.stride(0), _p(x), x.stride(0), _p(w),
                               _p(mean), _p(rstd), _p(out), out.stride(0), _p(dres),
                               dres.stride(0) if dres is not None else 0, _p(dw), _p(db), _p(dsum), int(accumulate),
                               float(drop[0]), int(drop[1]) & 0xFFFFFFFF, _p(out_drop),
                               out_drop.stride(0) if out_drop is not None else 0, _p(ws), wsb, _stream()),
          "capk_layernorm_bwd")
    _hold(ws)
    return out


# -------------------------------------------------------------- attention ---
class HeadView:
    """A [B, N, H*hd] token view inside a larger buffer: base tensor + offsets (elements)."""

    __slots__ = ("t", "off", "bs", "rs")

    def __init__(self, t, off, bs, rs):
        self.t, self.off, self.bs, self.rs = t, off, bs, rs

    def ptr(self):
        return self.t.data_ptr() + self.off * self.t.element_size()


def attention_fwd(q, k, v, o, B, H, Nq, Nk, hd, scale, causal=False, key_pad=None, drop=NO_DROP):
    """q/k/v/o: HeadView.  Returns lse [B,H,Nq] fp32."""
    lse = torch.empty(B, H, Nq, dtype=torch.float32, device=q.t.device)
    kp = None if key_pad is None else key_pad.to(torch.uint8).contiguous()
    check(lib().capk_attention_fwd(dtype_code(q.t), B, H, Nq, Nk, hd, float(scale), int(causal),
                                   q.ptr(), q.bs, q.rs, k.ptr(), k.bs, k.rs, v.ptr(), v.bs, v.rs, _p(kp),
                                   o.ptr(), o.bs, o.rs, _p(lse), float(drop[0]), int(drop[1]) & 0xFFFFFFFF,
                                   _stream()), "capk_attention_fwd")
    return lse, kp


def attention_decode_rows(q, k, v, o, rows, B, H, Nq, Nk, hd, scale, lse=None):
    """Decode step over a beam-history table (capk_attention_decode_rows): key j < Nk-1 of batch
    row b is read from K/V row rows[b, j] (int32 [B, ld]), the last key from row b."""
    if lse is None:
        lse = torch.empty(B, H, Nq, dtype=torch.float32, device=q.t.device)
    if rows.dtype != torch.int32 or rows.dim() != 2 or rows.stride(1) != 1 or rows.shape[0] != B:
        raise ValueError("attention_decode_rows: rows must be int32 [B, ld] with unit column stride")
    check(lib().capk_attention_decode_rows(dtype_code(q.t), B, H, Nq, Nk, hd, float(scale), q.ptr(), q.bs, q.rs,
                                           k.ptr(), k.bs, k.rs, v.ptr(), v.bs, v.rs, rows.data_ptr(), rows.stride(0),
                                           o.ptr(), o.bs, o.rs, _p(lse), _stream()), "capk_attention_decode_rows")
    return lse


def attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Nq, Nk, hd, scale, causal=False, key_pad_u8=None,
                  drop=NO_DROP):
    check(lib().capk_attention_bwd(dtype_code(q.t), B, H, Nq, Nk, hd, float(scale), int(causal),
                                   q.ptr(), q.bs, q.rs, k.ptr(), k.bs, k.rs, v.ptr(), v.bs, v.rs,
                                   _p(key_pad_u8), o.ptr(), o.bs, o.rs, do.ptr(), do.bs, do.rs, _p(lse),
                                   dq.ptr(), dq.bs, dq.rs, dk.ptr(), dk.bs, dk.rs, dv.ptr(), dv.bs, dv.rs,
                                   float(drop[0]), int(drop[1]) & 0xFFFFFFFF, _stream()), "capk_attention_bwd")


def attention_bwd_bias(q, k, v, o, do, lse, dq, dk, dv, B, H, Nq, Nk, hd, scale, dbias, *, causal=False,
                       key_pad_u8=None, drop=NO_DROP, accumulate=False):
    """attention_bwd + the fused QKV bias gradient: dbias [3*H*hd] fp32 (+)= column sums of dQ | dK | dV
    (capk_attention_bwd_bias)."""
    _need_gpu(dbias)
    L = lib()
    wsb = L.capk_attention_bwd_bias_workspace(B, H, Nq, Nk, hd)
    ws = _ws(wsb, q.t.device)
    check(L.capk_attention_bwd_bias(dtype_code(q.t), B, H, Nq, Nk, hd, float(scale), int(causal),
                                    q.ptr(), q.bs, q.rs, k.ptr(), k.bs, k.rs, v.ptr(), v.bs, v.rs,
                                    _p(key_pad_u8), o.ptr(), o.bs, o.rs, do.ptr(), do.bs, do.rs, _p(lse),
                                    dq.ptr(), dq.bs, dq.rs, dk.ptr(), dk.bs, dk.rs, dv.ptr(), dv.bs, dv.rs,
                                    float(drop[0]), int(drop[1]) & 0xFFFFFFFF, _p(dbias), int(accumulate), _p(ws), wsb,
                                    _stream()), "capk_attention_bwd_bias")
    _hold(ws)


# ------------------------------------------------------ embeddings / misc ---
def patchify(images, P, out_dtype):
    B, C, H, W = images.shape
    _need_gpu(images)
    out = torch.empty(B * (H // P) * (W // P), C * P * P, dtype=out_dtype, device=images.device)
    img = images.contiguous().float()
    check(lib().capk_patchify(_DT[out_dtype], B, C, H, W, P, _p(img), _p(out), _stream()), "capk_patchify")
    return out


def vit_assemble(patch_out, cls, pos, B, Np, D):
    x = torch.empty(B * (Np + 1), D, dtype=patch_out.dtype, device=patch_out.device)
    check(lib().capk_vit_assemble(dtype_code(patch_out), B, Np, D, _p(patch_out), _p(cls), _p(pos), _p(x),
                                  _stream()), "capk_vit_assemble")
    return x


def vit_assemble_bwd(dx, B, Np, D, dcls, dpos):
    L = lib()
    dpatch = torch.empty(B * Np, D, dtype=dx.dtype, device=dx.device)
    wsb = L.capk_vit_assemble_bwd_workspace(B, Np, D)
    ws = _ws(wsb, dx.device)
    check(L.capk_vit_assemble_bwd(dtype_code(dx), B, Np, D, _p(dx), _p(dpatch), _p(dcls), _p(dpos), _p(ws), wsb,
                                  _stream()), "capk_vit_assemble_bwd")
    return dpatch


def embedding_fwd(ids, table, pos, pos_offset, out_dtype, drop=NO_DROP):
    B, T = ids.shape
    D = table.shape[1]
    out = torch.empty(B * T, D, dtype=out_dtype, device=table.device)
    check(lib().capk_embedding_fwd(_DT[out_dtype], B, T, D, _p(ids), _p(table), _p(pos), int(pos_offset),
                                   float(drop[0]), int(drop[1]) & 0xFFFFFFFF, _p(out), _stream()),
          "capk_embedding_fwd")
    return out


def embedding_bwd(ids, dout, padding_idx, dtable, dpos, pos_offset=0, drop=NO_DROP):
    B, T = ids.shape
    D = dout.shape[1]
    check(lib().capk_embedding_bwd(dtype_code(dout), B, T, D, _p(ids), _p(dout),
                                   -1 if padding_idx is None else int(padding_idx), _p(dtable), _p(dpos),
                                   int(pos_offset), float(drop[0]), int(drop[1]) & 0xFFFFFFFF, _stream()),
          "capk_embedding_bwd")


def shifted_ce(logits2d, targets, B, T, V, ignore_index, *, want_loss=True, dlogits=None, grad_scale=None,
               row_weight=None):
    """loss fp32 [2] = (mean, count) if want_loss; fills dlogits (times *grad_scale, a device scalar).
    row_weight (fp32 [B], optional): per-sample weight (SCST advantage)."""
    L = lib()
    loss = torch.empty(2, dtype=torch.float32, device=logits2d.device) if want_loss else None
    wsb = L.capk_shifted_ce_workspace(B, T)
    ws = _ws(wsb, logits2d.device)
    if row_weight is None:
        check(L.capk_shifted_ce(dtype_code(logits2d), B, T, V, logits2d.stride(0), _p(logits2d), _p(targets),
                                int(ignore_index), _p(grad_scale), _p(loss), _p(dlogits), _p(ws), wsb, _stream()),
              "capk_shifted_ce")
    else:
        check(L.capk_shifted_ce_weighted(dtype_code(logits2d), B, T, V, logits2d.stride(0), _p(logits2d),
                                         _p(targets), int(ignore_index), _p(row_weight), _p(grad_scale), _p(loss),
                                         _p(dlogits), _p(ws), wsb, _stream()), "capk_shifted_ce_weighted")
    return loss


def sample_rows(logits, V, seed, step, out, logp=None):
    """out[r] (int64 view, any stride) ~ Categorical(softmax(logits[r, :V])) with the counter-based uniform.
    seed: an int, or a 1-element int32 device tensor read by the kernel (graph replay)."""
    if torch.is_tensor(seed):
        _need_gpu(seed)
        check(lib().capk_sample_rows_dev(dtype_code(logits), logits.shape[0], V, logits.stride(0), _p(logits),
                                         _p(seed), int(step), _p(out), out.stride(0), _p(logp), _stream()),
              "capk_sample_rows_dev")
        return out
    check(lib().capk_sample_rows(dtype_code(logits), logits.shape[0], V, logits.stride(0), _p(logits),
                                 int(seed) & 0xFFFFFFFF, int(step), _p(out), out.stride(0), _p(logp), _stream()),
          "capk_sample_rows")
    return out


def dropout_mask(n, p, seed, offset=0, device="cuda"):
    """uint8 [n]: the keep mask the kernels use for (p, seed) at indices offset..offset+n-1."""
    out = torch.empty(n, dtype=torch.uint8, device=device)
    check(lib().capk_dropout_mask(int(n), int(offset), float(p), int(seed) & 0xFFFFFFFF, _p(out), _stream()),
          "capk_dropout_mask")
    return out


def zero_gap_rows(t, B, rpb, S):
    """Zero rows b * rpb + j (S <= j < rpb) of a contiguous 2-D buffer (capk_zero_gap_rows)."""
    check(lib().capk_zero_gap_rows(_p(t), t.stride(0) * t.element_size(), t.shape[1] * t.element_size(), int(B),
                                   int(rpb), int(S), t.shape[0], _stream()), "capk_zero_gap_rows")
    return t


def zero_(t):
    check(lib().capk_zero(_p(t), t.numel() * t.element_size(), _stream()), "capk_zero")
    return t


def cast(x, out):
    check(lib().capk_cast(dtype_code(x), dtype_code(out), x.numel(), _p(x), _p(out), _stream()), "capk_cast")
    return out


def copy_rows(x, out):
    rows, cols = x.shape
    check(lib().capk_copy_rows(dtype_code(x), rows, cols, _p(x), x.stride(0), _p(out), out.stride(0), _stream()),
          "capk_copy_rows")
    return out


def act_bwd(dy, aux, act, out=None):
    if out is None:
        out = torch.empty_like(dy)
    check(lib().capk_act_bwd(dtype_code(dy), dy.numel(), int(act), _p(dy), _p(aux), _p(out), _stream()),
          "capk_act_bwd")
    return out


def adamw(param, grad, m, v, param_bf16, lr, wd, beta1, beta2, eps, step):
    if param_bf16 is not None:
        WT.join(param_bf16.device)  # transposes of the previous weights may still read the shadow
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    check(lib().capk_adamw(param.numel(), _p(param), _p(grad), _p(m), _p(v), _p(param_bf16), float(lr), float(wd),
                           float(beta1), float(beta2), float(eps), float(bc1), float(bc2), _stream()), "capk_adamw")
    if param_bf16 is not None:
        WT.weights_changed()  # a bf16 shadow changed: the K-major dX copies are stale


# ---------------------------------------------------------- Conv1D (GPT-2) ---
def conv1d(x, w, b=None, *, out=None, residual=None, act=0, preact=None, drop=NO_DROP):
    """HF Conv1D: y = dropout(act(x @ W + b)) + residual with W [in, out] row-major
    (transformers/pytorch_utils.py Conv1D; GPT-2 c_attn/c_proj/c_fc): the weight is
    the GEMM's N-major B operand, so no transpose is materialised."""
    M, K = x.shape
    N = w.shape[1]
    if out is None:
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    f8 = _fp8_route(x, w, M, N, K, act, True)
    if f8 is not None:
        return _linear_f8(x, f8[0], f8[1], out, b, residual, act, preact, drop)
    gemm(x, True, w, False, M, N, K, out, lda=x.stride(0), ldb=w.stride(0), ldc=out.stride(0), bias=b,
         residual=residual, ldr=residual.stride(0) if residual is not None else 0, act=act, preact=preact,
         ldx=preact.stride(0) if preact is not None else 0, drop=drop)
    return out


def conv1d_dx(dy, w, *, out=None, act_bwd=0, aux=None, beta=0.0):
    """dX[M, in] = dY[M, out] @ W[in, out]^T (optionally * act'(aux))."""
    M, N = dy.shape
    K = w.shape[0]
    if out is None:
        out = torch.empty(M, K, dtype=dy.dtype, device=dy.device)
    gemm(dy, True, w, True, M, K, N, out, lda=dy.stride(0), ldb=w.stride(0), ldc=out.stride(0), beta=beta,
         act=(ACT_BWD | act_bwd) if act_bwd else 0, aux=aux, ldx=aux.stride(0) if aux is not None else 0)
    return out


def gather_rows(x, idx, y, groups, rows, cols, ldx, gsx, ldy, gsy, x_off=0, y_off=0):
    """y[g][r] = x[g][idx[r]] (element offsets x_off / y_off into x / y)."""
    check(lib().capk_gather_rows(dtype_code(x), groups, rows, cols, idx.data_ptr(),
                                 x.data_ptr() + x_off * x.element_size(), ldx, gsx,
                                 y.data_ptr() + y_off * y.element_size(), ldy, gsy, _stream()), "capk_gather_rows")


# ------------------------------------------------------------------ Swin ----
def window_attn_fwd(qkv, C, H, ws, nw_img, scale, table, labels, out):
    """Swin window attention over window-ordered rows (capk.h); returns lse [nwin, H, N]."""
    _need_gpu(qkv, table, out)
    N = ws * ws
    nwin = qkv.shape[0] // N
    lse = torch.empty(nwin, H, N, dtype=torch.float32, device=qkv.device)
    check(lib().capk_window_attn_fwd(dtype_code(qkv), nwin, nw_img, ws, H, C // H, float(scale), _p(qkv),
                                     qkv.stride(0), C, _p(table), _p(labels), _p(out), out.stride(0), _p(lse),
                                     _stream()), "capk_window_attn_fwd")
    return lse


def window_attn_bwd(qkv, C, H, ws, nw_img, scale, table, labels, out, dout, lse, dqkv, dtable, accumulate=False):
    L = lib()
    N = ws * ws
    nwin = qkv.shape[0] // N
    wsb = L.capk_window_attn_bwd_workspace(nwin, ws, H)
    ws_t = _ws(wsb, qkv.device)
    check(L.capk_window_attn_bwd(dtype_code(qkv), nwin, nw_img, ws, H, C // H, float(scale), _p(qkv), qkv.stride(0),
                                 C, _p(table), _p(labels), _p(out), out.stride(0), _p(dout), dout.stride(0), _p(lse),
                                 _p(dqkv), dqkv.stride(0), _p(dtable), int(accumulate), _p(ws_t), wsb, _stream()),
          "capk_window_attn_bwd")


def rowscale_add(x, scale, group_rows, res=None, out=None):
    """out = res + x * scale[row // group_rows] (SwinDropPath's per-sample factor)."""
    rows, cols = x.shape
    if out is None:
        out = torch.empty_like(x)
    check(lib().capk_rowscale_add(dtype_code(x), rows, cols, _p(x), x.stride(0), _p(scale), int(group_rows),
                                  _p(res), res.stride(0) if res is not None else 0, _p(out), out.stride(0),
                                  _stream()), "capk_rowscale_add")
    return out


def dropout_apply(x, drop, out=None):
    """x * mask (GEMM-epilogue mask convention, index r*cols + c)."""
    if drop[0] <= 0:
        return x
    rows, cols = x.shape
    if out is None:
        out = torch.empty_like(x)
    check(lib().capk_dropout_apply(dtype_code(x), rows, cols, _p(x), x.stride(0), float(drop[0]),
                                   int(drop[1]) & 0xFFFFFFFF, _p(out), out.stride(0), _stream()),
          "capk_dropout_apply")
    return out


def add_rows(x, y, groups, rows, cols, gsx, ldx, nseg, seg, gsy, ldy, accumulate, x_off=0):
    check(lib().capk_add_rows(dtype_code(x), groups, rows, cols, x.data_ptr() + x_off * x.element_size(), gsx, ldx,
                              nseg, seg, _p(y), gsy, ldy, int(accumulate), _stream()), "capk_add_rows")


# ------------------------------------------------------------ LSTM decoder ---
def lstm_cell_fwd(gates, c_prev, c_out, h_out, act, h_drop=None, drop=NO_DROP):
    B, D = c_prev.shape
    check(lib().capk_lstm_cell_fwd(dtype_code(gates), B, D, _p(gates), gates.stride(0), _p(c_prev), _p(c_out),
                                   _p(h_out), h_out.stride(0), _p(h_drop), h_drop.stride(0) if h_drop is not None else 0,
                                   _p(act), float(drop[0]), int(drop[1]) & 0xFFFFFFFF, _stream()), "capk_lstm_cell_fwd")


def lstm_cell_bwd(act, c_prev, dh, dc, dgates):
    B, D = c_prev.shape
    check(lib().capk_lstm_cell_bwd(dtype_code(act), B, D, _p(act), _p(c_prev), _p(dh), dh.stride(0), _p(dc),
                                   _p(dgates), _stream()), "capk_lstm_cell_bwd")


def pair_slabs_plan(M, N, K):
    """(split count, fp32 elements) of capk_gemm_pair_slabs' slabs for an (M, N, K) product."""
    s = ctypes.c_int(0)
    nbytes = lib().capk_gemm_pair_workspace(M, N, K, ctypes.byref(s))
    return s.value, nbytes // 4


def gemm_pair_slabs(M, N, K, A, lda, B, ldb, b_kmajor, ws, *, A2=None, lda2=0, B2=None, ldb2=0, k1=0, n1=0):
    """Two-segment bf16 product into fp32 split-K slabs ws[s][M][N] (capk.h): K seam k1
    ([A | A2] [B | B2]^T) or N seam n1 (C[:, :n1] = A B^T, C[:, n1:] = A B2^T).  Returns
    the split count."""
    _need_gpu(A, B, B2, ws)
    L = lib()
    s = ctypes.c_int(0)
    timed = GEMM_TIMER.active()
    if timed:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    check(L.capk_gemm_pair_slabs(M, N, K, _p(A), lda, 1, _p(B), ldb, int(b_kmajor), _p(A2), lda2, _p(B2), ldb2,
                                 int(k1), int(n1), _p(ws), ws.numel() * ws.element_size(), ctypes.byref(s),
                                 _stream()), "capk_gemm_pair_slabs")
    if timed:
        ev1.record()
        # operands read once, the slabs written once
        nbytes = A.element_size() * (M * K + N * K) + 4 * s.value * M * N
        GEMM_TIMER.records.append((ev0, ev1, 2.0 * M * N * K, dtype_code(A), nbytes, 0))
    return s.value


# Decode steps: a GEMM whose output only feeds a LayerNorm (and the residual stream) writes
# split-K slabs that the LayerNorm sums (capk_layernorm_fwd_slabs), bit-identical to the
# product + reduce + LayerNorm launches it replaces.  CAPK_DECODE_SLABS=0: the separate route.
DECODE_SLABS = os.environ.get("CAPK_DECODE_SLABS", "1") != "0"


def product_ln(x, w, conv1d_weight, b, residual, ln_w, ln_b, eps, *, keep=False):
    """(LayerNorm(s), s or None) for s = x W^T + b + residual (nn.Linear weight [out, in]) or
    x W + b + residual (conv1d_weight: HF Conv1D [in, out]); s is materialised only with keep
    (the pre-LN residual stream).  Products that take the fp8 route, non-bf16 inputs and
    shapes outside the slab kernel's K % 64 take the separate launches."""
    M, K = x.shape
    N = w.shape[1] if conv1d_weight else w.shape[0]
    if (not DECODE_SLABS or x.dtype != torch.bfloat16 or K % 64 or N % 8 or N > 2048 or x.stride(0) % 8
            or _fp8_route(x, w, M, N, K, 0, conv1d_weight) is not None):
        s = (conv1d if conv1d_weight else linear)(x, w, b, residual=residual)
        return layernorm_fwd(s, ln_w, ln_b, eps)[0], s
    L = lib()
    sp = ctypes.c_int(0)
    ws = _ws(L.capk_gemm_slabs_workspace(M, N, K, ctypes.byref(sp)), x.device).view(torch.float32)
    splits = gemm_pair_slabs(M, N, K, x, x.stride(0), w, w.stride(0), not conv1d_weight, ws)
    y = torch.empty(M, N, dtype=x.dtype, device=x.device)
    s = torch.empty(M, N, dtype=x.dtype, device=x.device) if keep else None
    check(L.capk_layernorm_fwd_slabs(M, N, _p(ws), splits, _p(b), _p(residual),
                                     residual.stride(0) if residual is not None else 0, _p(s), N, _p(ln_w), _p(ln_b),
                                     float(eps), _p(y), N, _stream()), "capk_layernorm_fwd_slabs")
    return y, s


def lstm_cell_fwd_slabs(ws, splits, ldw, bias_a, bias_b, res, c_prev, c_out, h_out, act, h_drop=None, drop=NO_DROP):
    B, D = c_prev.shape
    check(lib().capk_lstm_cell_fwd_slabs(B, D, _p(ws), int(splits), ldw, _p(bias_a), _p(bias_b), _p(res),
                                         res.stride(0) if res is not None else 0, _p(c_prev), _p(c_out), _p(h_out),
                                         h_out.stride(0), _p(h_drop), h_drop.stride(0) if h_drop is not None else 0,
                                         _p(act), float(drop[0]), int(drop[1]) & 0xFFFFFFFF, _stream()),
          "capk_lstm_cell_fwd_slabs")


def lstm_cell_bwd_slabs(act, c_prev, dc, dgates, *, dh=None, up=None, drop=NO_DROP, rec=None):
    """up / rec: (slab tensor, splits, ld[, col]) -- the layer above's input-gradient slabs
    (columns 0:D, under the forward's dropout mask) and this layer's recurrent slabs."""
    B, D = c_prev.shape
    uw, us, ul = up if up is not None else (None, 0, 0)
    rw, rs, rl, rc = rec if rec is not None else (None, 0, 0, 0)
    check(lib().capk_lstm_cell_bwd_slabs(B, D, _p(act), _p(c_prev), _p(dh), dh.stride(0) if dh is not None else 0,
                                         _p(uw), int(us), ul, float(drop[0]), int(drop[1]) & 0xFFFFFFFF, _p(rw),
                                         int(rs), rl, int(rc), _p(dc), _p(dgates), _stream()),
          "capk_lstm_cell_bwd_slabs")


def slab_sum(ws, splits, M, ldw, col0, out, res=None):
    """out [M, ncols] bf16 view = sum over the splits of ws[s][:, col0:col0+ncols] (+ res)."""
    check(lib().capk_slab_sum(M, out.shape[1], _p(ws), int(splits), ldw, int(col0), _p(res),
                              res.stride(0) if res is not None else 0, _p(out), out.stride(0), _stream()),
          "capk_slab_sum")
    return out


def soft_attn_fwd(qp, kp, v, we, be, inv_temp, ctx, w_out, key_pad=None):
    """qp [B,D]; kp, v: [B,S,D] views (row strides free); ctx [B,D] view; w_out fp32 [B,S]."""
    B, S, D = kp.shape
    check(lib().capk_soft_attn_fwd(dtype_code(qp), B, S, D, _p(qp), qp.stride(0), _p(kp), kp.stride(0), kp.stride(1),
                                   _p(v), v.stride(0), v.stride(1), _p(we), _p(be), float(inv_temp), _p(key_pad),
                                   _p(ctx), ctx.stride(0), _p(w_out), _stream()), "capk_soft_attn_fwd")


def soft_attn_bwd(qp, kp, v, we, inv_temp, w, dctx, dqp, dkp, dv, dwe_part, dbe_part, dw_in=None):
    B, S, D = kp.shape
    check(lib().capk_soft_attn_bwd(dtype_code(qp), B, S, D, _p(qp), qp.stride(0), _p(kp), kp.stride(0), kp.stride(1),
                                   _p(v), v.stride(0), v.stride(1), _p(we), float(inv_temp), _p(w), _p(dctx),
                                   dctx.stride(0), _p(dw_in), _p(dqp), dqp.stride(0), _p(dkp), _p(dv), _p(dwe_part),
                                   _p(dbe_part), _stream()), "capk_soft_attn_bwd")


def soft_attn_bwd_step(qp, kp, v, we, inv_temp, w, dctx, dqp, dwe_part, dbe_part, de_out, dctx_out, dw_in=None):
    """soft_attn_bwd without the per-step dkp / dv updates: stashes de [B,S] and dctx [B,D]."""
    B, S, D = kp.shape
    check(lib().capk_soft_attn_bwd_step(dtype_code(qp), B, S, D, _p(qp), qp.stride(0), _p(kp), kp.stride(0),
                                        kp.stride(1), _p(v), v.stride(0), v.stride(1), _p(we), float(inv_temp), _p(w),
                                        _p(dctx), dctx.stride(0), _p(dw_in), _p(dqp), dqp.stride(0), _p(dwe_part),
                                        _p(dbe_part), _p(de_out), _p(dctx_out), _stream()), "capk_soft_attn_bwd_step")


def soft_attn_kv_grad(qp_all, kp, we, de_all, w_all, dctx_all, dkp, dv=None):
    """dkp (and dv) [B,S,D] fp32 written from the per-step stashes (capk.h)."""
    steps, B, D = qp_all.shape
    S = kp.shape[1]
    check(lib().capk_soft_attn_kv_grad(dtype_code(qp_all), steps, B, S, D, _p(qp_all), _p(kp), kp.stride(0),
                                       kp.stride(1), _p(we), _p(de_all), _p(w_all), _p(dctx_all), _p(dkp), _p(dv),
                                       _stream()), "capk_soft_attn_kv_grad")


def argmax_rows(x, V, out):
    """out[r] (int64 view, any stride) = argmax(x[r, :V])."""
    check(lib().capk_argmax_rows(dtype_code(x), x.shape[0], V, x.stride(0), _p(x), _p(out), out.stride(0), _stream()),
          "capk_argmax_rows")
    return out


# ------------------------------------------------ attention-module gates ---
def ew_mul(a, b, out):
    rows, cols = a.shape
    check(lib().capk_ew_mul(dtype_code(a), rows, cols, _p(a), a.stride(0), _p(b), b.stride(0), _p(out), out.stride(0),
                            _stream()), "capk_ew_mul")
    return out


def tanh_gate_fwd(c, g, out):
    rows, cols = g.shape
    check(lib().capk_tanh_gate_fwd(dtype_code(g), rows, cols, _p(c), c.stride(0), _p(g), g.stride(0), _p(out),
                                   out.stride(0), _stream()), "capk_tanh_gate_fwd")
    return out


def tanh_gate_bwd(c, g, dout, dg, dc):
    rows, cols = g.shape
    check(lib().capk_tanh_gate_bwd(dtype_code(g), rows, cols, _p(c), c.stride(0), _p(g), g.stride(0), _p(dout),
                                   dout.stride(0), _p(dg), dg.stride(0), _p(dc), dc.stride(0), _stream()),
          "capk_tanh_gate_bwd")


def gate_mix_fwd(ctx, s, wa, ba, beta, out):
    B, D = ctx.shape
    check(lib().capk_gate_mix_fwd(dtype_code(ctx), B, D, _p(ctx), ctx.stride(0), _p(s), s.stride(0), _p(wa), _p(ba),
                                  _p(beta), _p(out), out.stride(0), _stream()), "capk_gate_mix_fwd")
    return out


def gate_mix_bwd(ctx, s, wa, beta, dout, dctx, ds, dwa, dba):
    B, D = ctx.shape
    check(lib().capk_gate_mix_bwd(dtype_code(ctx), B, D, _p(ctx), ctx.stride(0), _p(s), s.stride(0), _p(wa), _p(beta),
                                  _p(dout), dout.stride(0), _p(dctx), dctx.stride(0), _p(ds), ds.stride(0), _p(dwa),
                                  _p(dba), _stream()), "capk_gate_mix_bwd")


def attention_probs_mean(q, k, lse, B, H, Nq, Nk, hd, scale, out, key_pad=None):
    check(lib().capk_attention_probs_mean(dtype_code(q.t), B, H, Nq, Nk, hd, float(scale), q.ptr(), q.bs, q.rs,
                                          k.ptr(), k.bs, k.rs, _p(key_pad), _p(lse), _p(out), _stream()),
          "capk_attention_probs_mean")
    return out


def attention_probs_mean_bwd(q, k, lse, dw, dq, dk, B, H, Nq, Nk, hd, scale, key_pad=None):
    """Gradient of attention_probs_mean: dw fp32 [B, Nq, Nk] contiguous; ACCUMULATES into dq
    (HeadView, model dtype) and dk (HeadView over an fp32 buffer)."""
    if dw.dtype != torch.float32 or not dw.is_contiguous() or dw.numel() != B * Nq * Nk:
        raise ValueError("attention_probs_mean_bwd: dw must be contiguous fp32 [B, Nq, Nk]")
    if dk.t.dtype != torch.float32:
        raise ValueError("attention_probs_mean_bwd: dk accumulates in fp32")
    check(lib().capk_attention_probs_mean_bwd(dtype_code(q.t), B, H, Nq, Nk, hd, float(scale), q.ptr(), q.bs, q.rs,
                                              k.ptr(), k.bs, k.rs, _p(key_pad), _p(lse), _p(dw), dq.ptr(), dq.bs,
                                              dq.rs, dk.ptr(), dk.bs, dk.rs, _stream()),
          "capk_attention_probs_mean_bwd")


# ------------------------------------------------- convolutional encoder (A3) ---
def conv_out_hw(H, W, k, stride, pad):
    return (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1


def im2col(x, B, H, W, C, k, stride, pad, Kp, out_dtype, strides=None, out=None):
    """Channels-last im2col panel [B*OH*OW, Kp] (k order kh, kw, c).  `strides` =
    element strides (sb, sh, sw, sc) of x; default = contiguous NHWC rows."""
    _need_gpu(x)
    OH, OW = conv_out_hw(H, W, k, stride, pad)
    if strides is None:
        strides = (H * W * C, W * C, C, 1)
    if out is None:
        out = torch.empty(B * OH * OW, Kp, dtype=out_dtype, device=x.device)
    check(lib().capk_im2col(dtype_code(x), dtype_code(out), B, H, W, C, *[int(s) for s in strides], k, k, stride,
                            pad, OH, OW, Kp, _p(x), _p(out), _stream()), "capk_im2col")
    return out


def col2im(dcol, dx, B, H, W, C, k, stride, pad, Kp, beta=0.0):
    OH, OW = conv_out_hw(H, W, k, stride, pad)
    check(lib().capk_col2im(dtype_code(dcol), B, H, W, C, k, k, stride, pad, OH, OW, Kp, _p(dcol), _p(dx),
                            float(beta), _stream()), "capk_col2im")
    return dx


def _bn_ws(M, C, device):
    return _ws(lib().capk_bn_workspace(M, C), device)


def bn_stats(x, eps, momentum, running_mean=None, running_var=None, num_batches_tracked=None):
    """Training-mode BatchNorm statistics of the rows of x [M, C]: (mean, rstd) fp32; the
    running buffers and the int64 batch counter (all optional) are updated in the launch."""
    _need_gpu(x)
    M, C = x.shape
    mean = torch.empty(C, dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    L = lib()
    wsb = L.capk_bn_workspace(M, C)
    ws = _ws(wsb, x.device)
    check(L.capk_bn_stats(dtype_code(x), M, C, _p(x), x.stride(0), float(eps), float(momentum), _p(mean), _p(rstd),
                          _p(running_mean), _p(running_var), _p(num_batches_tracked), _p(ws), wsb, _stream()),
          "capk_bn_stats")
    return mean, rstd


def bn_eval_stats(running_mean, running_var, eps):
    C = running_mean.numel()
    mean = torch.empty(C, dtype=torch.float32, device=running_mean.device)
    rstd = torch.empty_like(mean)
    check(lib().capk_bn_eval_stats(C, _p(running_mean), _p(running_var), float(eps), _p(mean), _p(rstd), _stream()),
          "capk_bn_eval_stats")
    return mean, rstd


def bn_apply(x, mean, rstd, gamma, beta, *, residual=None, relu=False, out=None):
    M, C = x.shape
    if out is None:
        out = torch.empty_like(x)
    check(lib().capk_bn_apply(dtype_code(x), M, C, _p(x), x.stride(0), _p(mean), _p(rstd), _p(gamma), _p(beta),
                              _p(residual), residual.stride(0) if residual is not None else 0, int(relu), _p(out),
                              out.stride(0), _stream()), "capk_bn_apply")
    return out


def bn_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, *, y_mask=None, dx=None, beta_acc=0.0, dz_out=None,
           accumulate=False, batch_stats=True, relu_beta=None):
    """BatchNorm backward (training statistics): dgamma/dbeta written (or added), dx
    (optional, += with beta_acc), dz_out (optional) = dy * [y_mask > 0]; relu_beta (the
    BatchNorm's beta) instead of y_mask: the mask of its own ReLU output, recomputed from x."""
    L = lib()
    M, C = x.shape
    wsb = L.capk_bn_workspace(M, C)
    ws = _ws(wsb, x.device)
    check(L.capk_bn_bwd(dtype_code(x), M, C, _p(dy), dy.stride(0), _p(y_mask),
                        y_mask.stride(0) if y_mask is not None else 0, _p(x), x.stride(0), _p(mean), _p(rstd),
                        _p(gamma), _p(relu_beta), _p(dgamma), _p(dbeta), int(accumulate), _p(dx),
                        dx.stride(0) if dx is not None else 0,
                        float(beta_acc), _p(dz_out), dz_out.stride(0) if dz_out is not None else 0,
                        int(batch_stats), _p(ws), wsb,
                        _stream()), "capk_bn_bwd")
    return dx


def maxpool_fwd(x, B, H, W, C, k, stride, pad):
    OH, OW = conv_out_hw(H, W, k, stride, pad)
    y = torch.empty(B * OH * OW, C, dtype=x.dtype, device=x.device)
    idx = torch.empty(B * OH * OW, C, dtype=torch.uint8, device=x.device)
    check(lib().capk_maxpool_fwd(dtype_code(x), B, H, W, C, k, stride, pad, OH, OW, _p(x), _p(y), _p(idx),
                                 _stream()), "capk_maxpool_fwd")
    return y, idx, OH, OW


def maxpool_bwd(dy, idx, B, H, W, C, k, stride, pad):
    OH, OW = conv_out_hw(H, W, k, stride, pad)
    dx = torch.empty(B * H * W, C, dtype=dy.dtype, device=dy.device)
    check(lib().capk_maxpool_bwd(dtype_code(dy), B, H, W, C, k, stride, pad, OH, OW, _p(dy), _p(idx), _p(dx),
                                 _stream()), "capk_maxpool_bwd")
    return dx


def avgpool_fwd(x, B, H, W, C, OH, OW, out=None):
    if out is None:
        out = torch.empty(B * OH * OW, C, dtype=x.dtype, device=x.device)
    check(lib().capk_avgpool_fwd(dtype_code(x), B, H, W, C, OH, OW, _p(x), _p(out), out.stride(0), _stream()),
          "capk_avgpool_fwd")
    return out


def avgpool_bwd(dy, B, H, W, C, OH, OW, dx=None, beta=0.0):
    if dx is None:
        dx = torch.empty(B * H * W, C, dtype=dy.dtype, device=dy.device)
    check(lib().capk_avgpool_bwd(dtype_code(dy), B, H, W, C, OH, OW, _p(dy), dy.stride(0), _p(dx), float(beta),
                                 _stream()), "capk_avgpool_bwd")
    return dx


# ----------------------------------------------- legacy Show-Attend-Tell (A11) ---
def additive_attn_fwd(act, qp, kp, v, we, be, inv_temp, ctx, w_out, key_pad=None):
    """qp [B,D]; kp [B,S,D], v [B,S,Dv] views; ctx [B,Dv] view; w_out fp32 [B,S].
    act 0 = tanh energy (SoftAttention), 1 = ReLU energy (legacy decoder)."""
    B, S, D = kp.shape
    Dv = v.shape[2]
    check(lib().capk_additive_attn_fwd(dtype_code(qp), int(act), B, S, D, Dv, _p(qp), qp.stride(0), _p(kp),
                                       kp.stride(0), kp.stride(1), _p(v), v.stride(0), v.stride(1), _p(we), _p(be),
                                       float(inv_temp), _p(key_pad), _p(ctx), ctx.stride(0), _p(w_out), _stream()),
          "capk_additive_attn_fwd")


def additive_attn_bwd(act, qp, kp, v, we, inv_temp, w, dctx, dqp, dkp, dv, dwe_part, dbe_part, dw_in=None):
    B, S, D = kp.shape
    Dv = v.shape[2]
    check(lib().capk_additive_attn_bwd(dtype_code(qp), int(act), B, S, D, Dv, _p(qp), qp.stride(0), _p(kp),
                                       kp.stride(0), kp.stride(1), _p(v), v.stride(0), v.stride(1), _p(we),
                                       float(inv_temp), _p(w), _p(dctx), dctx.stride(0), _p(dw_in), _p(dqp),
                                       dqp.stride(0), _p(dkp), _p(dv), _p(dwe_part), _p(dbe_part), _stream()),
          "capk_additive_attn_bwd")


def attn_coverage_reg(alphas_tbs, grad_scale=None, loss_acc=None, coef=None):
    T, B, S = alphas_tbs.shape
    check(lib().capk_attn_coverage_reg(B, T, S, _p(alphas_tbs), _p(grad_scale), _p(loss_acc), _p(coef), _stream()),
          "capk_attn_coverage_reg")


def clamp_(x, lo, hi):
    check(lib().capk_clamp(x.numel(), _p(x), float(lo), float(hi), _stream()), "capk_clamp")
    return x


def mask_rows_by_length(x, lengths_i32):
    """x: [B, T, C] view (row stride x.stride(1), batch stride x.stride(0)); zero rows t >= len[b]."""
    B, T, C = x.shape
    check(lib().capk_mask_rows_by_length(dtype_code(x), B, T, C, _p(x), x.stride(1), x.stride(0), _p(lengths_i32),
                                         _stream()), "capk_mask_rows_by_length")
    return x
