"""Shared pieces of the capk model modules: precision, parameter access, and the
fused transformer building blocks (pre-/post-LN attention + MLP) expressed as
sequences of libcapk kernel launches with explicit backward passes.

Each block is a ``torch.autograd.Function`` whose backward writes parameter
gradients straight into the flat fp32 gradient buffer of the ParamStore
(``p._capk_grad``) and returns only the activation gradient; one parameter per
block is passed as an "anchor" input so autograd schedules the backward.
"""
import os

import torch
import torch.nn as nn

from .. import ops
from ..ops import HeadView


_SEED = [None]


def next_seed():
    """Fresh 32-bit dropout seed (host counter; no device sync).  Seeded from torch's
    initial seed so runs are reproducible under torch.manual_seed."""
    if _SEED[0] is None:
        _SEED[0] = (torch.initial_seed() * 0x9E3779B1) & 0xFFFFFFFF
    _SEED[0] = (_SEED[0] * 1664525 + 1013904223) & 0xFFFFFFFF
    return _SEED[0]


def compute_dtype(m):
    return getattr(m, "_capk_dtype", torch.bfloat16)


def W(p, dtype):
    """Weight as the kernels consume it: bf16 shadow in bf16 mode, fp32 master otherwise."""
    if dtype == torch.bfloat16:
        return p._capk_bf16
    return p.detach()


def G(p):
    return p._capk_grad


def mark(p):
    st = getattr(p, "_capk_store_ref", None)
    if st is not None:
        st.mark_written(p)


def set_precision(model, dtype):
    """'bf16' (throughput path) or 'fp32' (parity path) for every capk module."""
    if isinstance(dtype, str):
        dtype = {"bf16": torch.bfloat16, "fp32": torch.float32, "float32": torch.float32,
                 "bfloat16": torch.bfloat16}[dtype]
    for m in model.modules():
        m._capk_dtype = dtype
    return model


class CapkModule(nn.Module):
    """Base class: modules whose forward runs on libcapk kernels."""

    @property
    def cdtype(self):
        return compute_dtype(self)

    def _check_ready(self, p):
        if not hasattr(p, "_capk_grad"):
            raise RuntimeError("capk: parameters are not attached to a ParamStore; call "
                               "capk.prepare(model, device) before running the model")


# Weight-gradient side stream: a layer's dW = dY^T X (and its bias column sums) depends on
# nothing the rest of the backward produces, so the encoder layers issue it on a second HIP
# stream and the dX chain (attention backward, LayerNorm backward, column sums: memory- or
# latency-bound kernels that leave the MFMAs idle) proceeds on the compute stream meanwhile.
# join_dw() makes the compute stream wait before the gradients are read (the patch-embedding
# backward, the optimizer).  Opt-in (CAPK_DW_STREAM=1), and off under multi-rank DP (the
# bucketer launches a layer's all-reduce as soon as it is notified).  Measured on config 3 it
# gains 0.9 % per step, but the side-stream GEMMs share the CUs with the dX chain, so their
# launch durations stretch and the per-GEMM roofline reading falls 0.34 -> 0.26 of peak; the
# default keeps one stream ("tried and not kept").
DW_STREAM = os.environ.get("CAPK_DW_STREAM", "0") == "1"
_DW_SIDE = {}
_DW_PENDING = set()


def _dw_side_on():
    if not DW_STREAM:
        return False
    import torch.distributed as dist
    return not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1)


def join_dw(device=None):
    """Make the current stream wait for the weight gradients issued on the side stream."""
    for dev in list(_DW_PENDING):
        if device is None or dev == device:
            torch.cuda.current_stream(dev).wait_stream(_DW_SIDE[dev])
            _DW_PENDING.discard(dev)


def linear_bwd(dy, x, w_param, b_param, dtype, *, fused=None, need_dx=True, act_bwd=0, aux=None,
               dw_accumulate=False, drop=(0.0, 0), dsum=None, side_dw=False):
    """Backward of y = x W^T + b: dW, db into the grad buffer; returns dX (or None).
    dsum: with act_bwd, the column sums of the returned dX (the bias gradient of the Linear
    below the activation) are written there, fused into the activation pass.
    side_dw: dW / db on the weight-gradient side stream (see join_dw)."""
    if fused is not None:
        wmat, gw = fused[0].w(dtype), fused[0].grad
        gb = fused[1].grad if fused[1] is not None else None
    else:
        wmat, gw = W(w_param, dtype), G(w_param)
        gb = G(b_param) if b_param is not None else None
    if side_dw and dy.is_cuda and _dw_side_on():
        dev = dy.device
        side = _DW_SIDE.get(dev)
        if side is None:
            side = _DW_SIDE[dev] = torch.cuda.Stream(device=dev)
        if dev not in _DW_PENDING:
            # also join at the end of this backward pass, so that code reading the gradients
            # between backward() and the optimizer (clipping, a partially frozen encoder whose
            # embedding backward never runs, the end of a graph capture) sees them complete
            torch.autograd.Variable._execution_engine.queue_callback(lambda: join_dw(dev))
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            ops.linear_dw(dy, x, gw, accumulate=dw_accumulate)
            if gb is not None:
                ops.colsum(dy, gb, accumulate=dw_accumulate)
        dy.record_stream(side)  # the compute stream may free these before the side stream is done
        x.record_stream(side)
        _DW_PENDING.add(dev)
    else:
        ops.linear_dw(dy, x, gw, accumulate=dw_accumulate)
        if gb is not None:
            ops.colsum(dy, gb, accumulate=dw_accumulate)
    if not need_dx:
        return None
    return ops.linear_dx(dy, wmat, act_bwd=act_bwd, aux=aux, drop=drop, dsum=dsum)


def heads(buf, col_off, B, N, row_stride_rows=None):
    """HeadView over a [B*N, C] buffer for columns starting at col_off."""
    C = buf.shape[1]
    rs = C
    bs = (row_stride_rows if row_stride_rows is not None else N) * C
    return HeadView(buf, col_off, bs, rs)
