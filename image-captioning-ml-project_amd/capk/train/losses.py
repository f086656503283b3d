"""Caption loss — mirrors src/train/losses.py CombinedLoss (169-263) CE path.

The shifted cross entropy (logits[:, :-1] vs targets[:, 1:], ignore_index=pad,
mean over counted tokens; losses.py:236-247) runs as one libcapk kernel per
pass: forward computes row log-sum-exp + target logit; backward recomputes the
softmax and writes d(loss)/d(logits) scaled by the upstream gradient read on
the device (no host sync).  The contrastive / ITM terms are never activated by
the reference trainer and are out of scope here.
"""
import torch
import torch.nn as nn

from .. import ops


def _padded_base(logits):
    """capk decoders return logits as a [B,T,V] view of a zero-padded [B*T, Vp] buffer."""
    B, T, V = logits.shape
    base = logits._base
    if base is not None and base.dim() == 2 and base.shape[0] == B * T and base.is_contiguous() \
            and base.data_ptr() == logits.data_ptr() and logits.stride(1) == base.shape[1]:
        return base
    if logits.stride(2) == 1 and logits.stride(1) % 8 == 0 and logits.stride(0) == T * logits.stride(1):
        return logits.as_strided((B * T, logits.stride(1)), (logits.stride(1), 1))
    raise ValueError("capk CE needs [B,T,V] logits with a unit-stride, 8-aligned row layout")


def _lm_partials(base):
    """The softmax partials the decoder's LM head left on its padded logits buffer
    (ops.linear_lse), if they still describe it (the buffer not written since)."""
    info = getattr(base, "_capk_ce_part", None)
    if info is None or info[1] != base._version:
        return None
    return info[0]


class _ShiftedCEFn(torch.autograd.Function):
    """Forward: the loss from the LM head's softmax partials when the decoder left them
    (capk_ce_lse_fwd: no pass over the logits), else one capk_shifted_ce pass.  Backward: with the
    partials' row lse, one streaming pass that also writes the LM-head bias gradient the decoder
    registered on the buffer (capk_ce_lse_bwd); else capk_shifted_ce's gradient."""

    @staticmethod
    def forward(ctx, logits, targets, pad):
        B, T, V = logits.shape
        base = _padded_base(logits)
        targets = targets.contiguous()
        part = _lm_partials(base)
        if part is not None:
            loss, lse = ops.ce_lse_fwd(base, targets, B, T, V, pad, part)
            ctx.save_for_backward(targets, lse, loss)
        else:
            loss = ops.shifted_ce(base, targets, B, T, V, pad, want_loss=True)
            ctx.save_for_backward(targets)
        ctx.base = base
        ctx.dims = (B, T, V, pad)
        return loss[0]

    @staticmethod
    def backward(ctx, dloss):
        saved = ctx.saved_tensors
        B, T, V, pad = ctx.dims
        base = ctx.base
        ctx.base = None
        dbase = torch.empty_like(base)
        gs = dloss.reshape(1).float().contiguous()
        if len(saved) == 3:
            targets, lse, loss = saved
            dbias = getattr(base, "_capk_bias_grad", None)
            ops.ce_lse_bwd(base, targets, B, T, V, pad, lse, loss, gs, dbase, dbias)
            if dbias is not None:  # the decoder's LM-head backward then skips its column sums
                dbase._capk_bias_done = True
        else:
            ops.shifted_ce(base, saved[0], B, T, V, pad, want_loss=False, dlogits=dbase, grad_scale=gs)
        return dbase[:, :V].view(B, T, V), None, None


def shifted_cross_entropy(logits, targets, pad_token_id):
    return _ShiftedCEFn.apply(logits, targets, int(pad_token_id))


class CombinedLoss(nn.Module):
    def __init__(self, pad_token_id, use_contrastive=False, use_itm=False, contrastive_weight=0.1, itm_weight=0.1,
                 temperature=0.07, hidden_dim=768):
        super().__init__()
        if use_contrastive or use_itm:
            raise NotImplementedError("capk: contrastive/ITM losses are never activated by the reference trainer")
        self.pad_token_id = pad_token_id

    def forward(self, logits, targets, image_features=None, text_features=None):
        ce = shifted_cross_entropy(logits, targets, self.pad_token_id)
        return {"ce_loss": ce, "total_loss": ce}
