"""Swin Transformer image encoder on libcapk kernels (``SwinEncoder``,
src/models/encoders.py:140-182, on transformers 5.15 ``SwinModel``,
modeling_swin.py:167-900).

Module tree and parameter names mirror ``SwinModel`` (``embeddings.patch_embeddings.
projection``, ``embeddings.norm``, ``encoder.layers.{s}.blocks.{i}.attention.{q,k,v,o}_proj``,
``...attention.relative_position_bias.relative_position_bias_table``,
``...layernorm_before/after``, ``...mlp.fc1/fc2``, ``encoder.layers.{s}.downsample.
{norm,reduction}``, ``layernorm``), so reference checkpoints load unchanged.

MI355X formulation.  A Swin block is row-wise everywhere except its window attention,
and the cyclic shift + window_partition (and their inverses) are a permutation of the
token rows.  The residual stream is therefore kept in the *window order* of the block
that consumes it: one row gather (capk_gather_rows) moves it from one block's order to
the next (shifted <-> unshifted), the block runs on plain [rows, C] buffers
(LN, fused QKV GEMM, capk_window_attn_fwd with the relative-position bias and shift mask
computed in-kernel, O GEMM + residual, LN, FC1 + GELU, FC2 + residual), and
window_reverse / the reverse roll are never materialised.  Patch merging is one gather
(2x2 neighbours -> [rows/4, 4C]) + LN + GEMM.  The final LN, the optional projection
to feature_dim and the token mean (the reference's ``features.mean(dim=1)``) end the
encoder.  SwinDropPath (attention branch only, as in SwinLayer.forward) multiplies each
sample's branch by floor(keep + U)/keep with U drawn by torch's RNG (capk_rowscale_add).

Shapes whose resolution is not a multiple of the window (SwinLayer.maybe_pad) or odd at
a patch merge are not supported (the reference's 224 input never pads).
"""
import math

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from .._lib import ACT_GELU_ERF
from ..params import Fused, notify_final, store_of
from .common import G, CapkModule, W, linear_bwd
from .resnet import GK, WK, kernel_layout

_BASE = dict(image_size=224, patch_size=4, num_channels=3, window_size=7, mlp_ratio=4.0, qkv_bias=True,
             layer_norm_eps=1e-5, drop_path_rate=0.1)
SWIN_ARCHS = {
    # pretrained_model_name -> SwinConfig fields (random-init offline; load a checkpoint by name)
    "microsoft/swin-base-patch4-window7-224": dict(_BASE, embed_dim=128, depths=(2, 2, 18, 2),
                                                   num_heads=(4, 8, 16, 32)),
    "microsoft/swin-tiny-patch4-window7-224": dict(_BASE, embed_dim=96, depths=(2, 2, 6, 2),
                                                   num_heads=(3, 6, 12, 24)),
    "microsoft/swin-small-patch4-window7-224": dict(_BASE, embed_dim=96, depths=(2, 2, 18, 2),
                                                    num_heads=(3, 6, 12, 24)),
}


# ------------------------------------------------------------ row orders ----
def window_order(B, Hs, Ws, ws, shift):
    """Natural row (b*Hs*Ws + h*Ws + w) of window row r: the rows of
    window_partition(torch.roll(x, (-shift, -shift))) (modeling_swin.py:486-496, 617-626)."""
    nh, nw = Hs // ws, Ws // ws
    b, wh, ww, r, c = np.meshgrid(np.arange(B), np.arange(nh), np.arange(nw), np.arange(ws), np.arange(ws),
                                  indexing="ij")
    h = (wh * ws + r + shift) % Hs
    w = (ww * ws + c + shift) % Ws
    return (b * Hs * Ws + h * Ws + w).reshape(-1)


def shift_labels(Hs, Ws, ws, shift):
    """[nW, ws*ws] region ids of SwinLayer.get_attn_mask (modeling_swin.py:584-607): pairs
    with different ids get -100."""
    hh = np.arange(Hs)
    wv = np.arange(Ws)
    hr = (hh >= Hs - ws).astype(np.int64) + (hh >= Hs - shift)
    wr = (wv >= Ws - ws).astype(np.int64) + (wv >= Ws - shift)
    img = hr[:, None] * 3 + wr[None, :]
    nh, nw = Hs // ws, Ws // ws
    return img.reshape(nh, ws, nw, ws).transpose(0, 2, 1, 3).reshape(nh * nw, ws * ws)


def merge_order(B, Hs, Ws):
    """Source natural row of chunk k of merged row (b, i, j): SwinPatchMerging's
    cat([x[:, row::2, col::2] for col in (0, 1) for row in (0, 1)]) (modeling_swin.py:309-326)."""
    b, i, j, k = np.meshgrid(np.arange(B), np.arange(Hs // 2), np.arange(Ws // 2), np.arange(4), indexing="ij")
    dr, dc = k % 2, k // 2
    return (b * Hs * Ws + (2 * i + dr) * Ws + (2 * j + dc)).reshape(-1)


class _OrderCache:
    """Device int32 index maps, built once per geometry."""

    def __init__(self):
        self.maps = {}

    def get(self, key, fn, device):
        k = (key, str(device))
        if k not in self.maps:
            a = np.ascontiguousarray(fn(), dtype=np.int32)
            self.maps[k] = torch.from_numpy(a).to(device)
        return self.maps[k]


_CACHE = _OrderCache()


def _inverse(p):
    inv = np.empty_like(p)
    inv[p] = np.arange(p.size, dtype=p.dtype)
    return inv


# ----------------------------------------------------------------- modules --
class _PatchEmbeddings(nn.Module):
    def __init__(self, a):
        super().__init__()
        P = a["patch_size"]
        self.projection = kernel_layout(nn.Conv2d(a["num_channels"], a["embed_dim"], P, P))


class _Embeddings(nn.Module):
    def __init__(self, a):
        super().__init__()
        self.patch_embeddings = _PatchEmbeddings(a)
        self.norm = nn.LayerNorm(a["embed_dim"])  # SwinEmbeddings.norm: default eps 1e-5


class _RelativePositionBias(nn.Module):
    def __init__(self, heads, ws):
        super().__init__()
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) ** 2, heads))


class _Attention(nn.Module):
    def __init__(self, d, heads, ws, qkv_bias):
        super().__init__()
        if not qkv_bias:
            raise NotImplementedError("capk Swin: qkv_bias=False")
        self.q_proj = nn.Linear(d, d)
        self.k_proj = nn.Linear(d, d)
        self.v_proj = nn.Linear(d, d)
        self.o_proj = nn.Linear(d, d)
        self.relative_position_bias = _RelativePositionBias(heads, ws)
        self.qkv_w = Fused([self.q_proj.weight, self.k_proj.weight, self.v_proj.weight])
        self.qkv_b = Fused([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias])

    def _capk_fused_groups(self):
        return [self.qkv_w, self.qkv_b]


class _MLP(nn.Module):
    def __init__(self, d, i):
        super().__init__()
        self.fc1 = nn.Linear(d, i)
        self.fc2 = nn.Linear(i, d)


class SwinLayer(CapkModule):
    """SwinLayer (modeling_swin.py:508-626)."""

    def __init__(self, a, dim, heads, shift, drop_path):
        super().__init__()
        self.heads = heads
        self.window_size = a["window_size"]
        self.shift_size = shift
        self.drop_path = drop_path
        self.eps = a["layer_norm_eps"]
        self.attention = _Attention(dim, heads, self.window_size, a["qkv_bias"])
        self.layernorm_before = nn.LayerNorm(dim, eps=self.eps)
        self.layernorm_after = nn.LayerNorm(dim, eps=self.eps)
        self.mlp = _MLP(dim, int(a["mlp_ratio"] * dim))

    def geometry(self, Hs, Ws):
        """(window, shift) after SwinLayer.set_shift_and_window_size (modeling_swin.py:576-582)."""
        ws, shift = self.window_size, self.shift_size
        if min(Hs, Ws) <= ws:
            ws, shift = min(Hs, Ws), 0
        if Hs % ws or Ws % ws:
            raise NotImplementedError(f"capk Swin: resolution {Hs}x{Ws} needs window padding (ws={ws})")
        return ws, shift


class _PatchMerging(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = nn.LayerNorm(4 * dim)


class SwinStage(nn.Module):
    def __init__(self, a, dim, depth, heads, dpr, downsample):
        super().__init__()
        ws = a["window_size"]
        self.blocks = nn.ModuleList([SwinLayer(a, dim, heads, 0 if i % 2 == 0 else ws // 2, dpr[i])
                                     for i in range(depth)])
        self.downsample = _PatchMerging(dim) if downsample else None


class _SwinEncoderStages(nn.Module):
    def __init__(self, a):
        super().__init__()
        depths = a["depths"]
        total = sum(depths)
        dpr = [a["drop_path_rate"] * i / max(total - 1, 1) for i in range(total)]  # SwinEncoder.__init__
        self.layers = nn.ModuleList()
        for s, d in enumerate(depths):
            self.layers.append(SwinStage(a, a["embed_dim"] * 2 ** s, d, a["num_heads"][s],
                                         dpr[sum(depths[:s]):sum(depths[:s + 1])], s < len(depths) - 1))


class CapkSwinModel(CapkModule):
    """SwinModel (modeling_swin.py:825-900); its AdaptiveAvgPool1d pooler has no parameters and
    its output is unused by the reference (encoders.py:165-172), so it is not built."""

    def __init__(self, arch):
        super().__init__()
        self.arch = dict(arch)
        self.num_features = arch["embed_dim"] * 2 ** (len(arch["depths"]) - 1)
        self.config = type("SwinArch", (), dict(arch, hidden_size=self.num_features))()
        self.embeddings = _Embeddings(arch)
        self.encoder = _SwinEncoderStages(arch)
        self.layernorm = nn.LayerNorm(self.num_features, eps=arch["layer_norm_eps"])
        self._init_weights()

    def _init_weights(self):
        # SwinPreTrainedModel._init_weights: normal(0.02) Linear/Conv weights, zero bias, LN 1/0,
        # zero relative-position tables
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                nn.init.normal_(m.weight, 0.0, 0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, _RelativePositionBias):
                nn.init.zeros_(m.relative_position_bias_table)

    def forward(self, images):
        """images [B,C,H,W] -> (normalised last hidden state [B*h*w, C_last] in natural row
        order, (B, h, w))."""
        a = self.arch
        B = images.shape[0]
        P = a["patch_size"]
        if images.shape[2] % P or images.shape[3] % P:
            raise NotImplementedError("capk Swin: image size must be a multiple of the patch size")
        Hs, Ws = images.shape[2] // P, images.shape[3] // P
        dev = images.device
        x = _SwinEmbedFn.apply(images, self.embeddings.patch_embeddings.projection.weight, self, B, Hs, Ws)
        cur = None  # key of the stream's row order (None: natural)
        for stage in self.encoder.layers:
            for blk in stage.blocks:
                ws, shift = blk.geometry(Hs, Ws)
                key = (B, Hs, Ws, ws, shift)
                if key != cur:
                    x = _reorder(x, cur, key, dev)
                    cur = key
                labels = None
                if shift > 0:
                    labels = _CACHE.get(("labels", Hs, Ws, ws, shift), lambda: shift_labels(Hs, Ws, ws, shift), dev)
                x = _SwinBlockFn.apply(x, blk.attention.o_proj.weight, blk, B, Hs * Ws, ws, labels)
            if stage.downsample is not None:
                if Hs % 2 or Ws % 2:
                    raise NotImplementedError("capk Swin: odd resolution at a patch merge needs padding")
                x = _merge(x, stage.downsample, cur, B, Hs, Ws, dev)
                cur = None
                Hs, Ws = Hs // 2, Ws // 2
        if cur is not None:
            x = _reorder(x, cur, None, dev)
        return x, (B, Hs, Ws)


def _natural_of(key):
    """Natural row of each row in the order `key` (None: identity)."""
    return window_order(*key)


def _reorder(x, cur, new, dev):
    """Move the stream from row order `cur` to `new` with one gather: row r of the result is
    row pos_cur[natural_new[r]] of x."""

    def fwd():
        nat = np.arange(x.shape[0]) if new is None else _natural_of(new)
        if cur is None:
            return nat
        return _inverse(_natural_of(cur))[nat]

    idx = _CACHE.get(("reorder", cur, new), fwd, dev)
    inv = _CACHE.get(("reorder_inv", cur, new), lambda: _inverse(fwd()), dev)
    return _GatherFn.apply(x, idx, inv)


def _merge(x, ds, cur, B, Hs, Ws, dev):
    def fwd():
        src = merge_order(B, Hs, Ws)
        return src if cur is None else _inverse(_natural_of(cur))[src]

    idx = _CACHE.get(("merge", cur, B, Hs, Ws), fwd, dev)
    inv = _CACHE.get(("merge_inv", cur, B, Hs, Ws), lambda: _inverse(fwd()), dev)
    return _MergeFn.apply(x, ds.reduction.weight, ds, idx, inv)


# --------------------------------------------------------------- functions --
def _gather(x, idx, rows_out):
    y = torch.empty(rows_out, x.shape[1], dtype=x.dtype, device=x.device)
    ops.gather_rows(x, idx, y, 1, rows_out, x.shape[1], x.stride(0), 0, y.stride(0), 0)
    return y


class _GatherFn(torch.autograd.Function):
    """y = x[idx] for a bijective row map (shift / window partition and their inverses)."""

    @staticmethod
    def forward(ctx, x, idx, inv):
        ctx.inv = inv
        return _gather(x, idx, idx.numel())

    @staticmethod
    def backward(ctx, dy):
        return _gather(dy.contiguous(), ctx.inv, ctx.inv.numel()), None, None


class _SwinEmbedFn(torch.autograd.Function):
    """SwinPatchEmbeddings (4x4/4 conv as im2col from NCHW + GEMM + bias) and SwinEmbeddings.norm
    (modeling_swin.py:219-286)."""

    @staticmethod
    def forward(ctx, images, anchor, m, B, Hs, Ws):
        dt = m.cdtype
        conv = m.embeddings.patch_embeddings.projection
        _, C, H, Wd = images.shape
        P = conv.kernel_size[0]
        images = images.contiguous()
        col = ops.im2col(images, B, H, Wd, C, P, P, 0, conv._capk_kp, dt, strides=(C * H * Wd, Wd, 1, H * Wd))
        pe = ops.linear(col, WK(conv.weight, dt), conv.bias.detach())
        ln = m.embeddings.norm
        x, mu, rs = ops.layernorm_fwd(pe, ln.weight.detach(), ln.bias.detach(), ln.eps)
        ctx.m = m
        ctx.saved = (col, pe, mu, rs)
        return x

    @staticmethod
    def backward(ctx, dx):
        m = ctx.m
        col, pe, mu, rs = ctx.saved
        ctx.saved = None
        ln = m.embeddings.norm
        dpe = ops.layernorm_bwd(dx.contiguous(), pe, ln.weight.detach(), mu, rs, G(ln.weight), G(ln.bias))
        conv = m.embeddings.patch_embeddings.projection
        ops.linear_dw(dpe, col, GK(conv.weight))
        ops.colsum(dpe, G(conv.bias))
        notify_final(store_of(m), all_except=[])  # the encoder's backward ends here
        return None, None, None, None, None, None


def _drop_path_scale(L, B, device):
    """SwinDropPath (modeling_swin.py:53-60): floor(keep + U) / keep per sample, or None."""
    if not L.training or L.drop_path <= 0.0:
        return None
    keep = 1.0 - L.drop_path
    u = torch.rand(B, dtype=torch.float32, device=device)
    return torch.floor(u + keep) / keep


class _SwinBlockFn(torch.autograd.Function):
    """SwinLayer.forward (modeling_swin.py:529-574) on window-ordered rows:
    x1 = x + drop_path(o_proj(window_attention(LN_before(x)))); y = x1 + fc2(GELU(fc1(LN_after(x1))))."""

    @staticmethod
    def forward(ctx, x, anchor, L, B, Limg, ws, labels):
        dt = L.cdtype
        C = x.shape[1]
        H = L.heads
        at = L.attention
        ln1, ln2, fc1, fc2 = L.layernorm_before, L.layernorm_after, L.mlp.fc1, L.mlp.fc2
        nW = Limg // (ws * ws)
        scale = (C // H) ** -0.5
        table = at.relative_position_bias.relative_position_bias_table.detach()
        h1, mu1, rs1 = ops.layernorm_fwd(x, ln1.weight.detach(), ln1.bias.detach(), L.eps)
        qkv = ops.linear(h1, at.qkv_w.w(dt), at.qkv_b.master)
        ctxo = torch.empty(x.shape[0], C, dtype=x.dtype, device=x.device)
        lse = ops.window_attn_fwd(qkv, C, H, ws, nW, scale, table, labels, ctxo)
        keep = _drop_path_scale(L, B, x.device)
        if keep is None:
            x1 = ops.linear(ctxo, W(at.o_proj.weight, dt), at.o_proj.bias.detach(), residual=x)
        else:
            a = ops.linear(ctxo, W(at.o_proj.weight, dt), at.o_proj.bias.detach())
            x1 = ops.rowscale_add(a, keep, Limg, res=x)
        h2, mu2, rs2 = ops.layernorm_fwd(x1, ln2.weight.detach(), ln2.bias.detach(), L.eps)
        f_pre = torch.empty(x.shape[0], fc1.weight.shape[0], dtype=x.dtype, device=x.device)
        f = ops.linear(h2, W(fc1.weight, dt), fc1.bias.detach(), act=ACT_GELU_ERF, preact=f_pre)
        y = ops.linear(f, W(fc2.weight, dt), fc2.bias.detach(), residual=x1)
        ctx.L, ctx.geo = L, (Limg, ws, nW, scale, labels)
        ctx.saved = (x, h1, mu1, rs1, qkv, ctxo, lse, keep, x1, h2, mu2, rs2, f_pre, f)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = ctx.L
        Limg, ws, nW, scale, labels = ctx.geo
        dt = L.cdtype
        x, h1, mu1, rs1, qkv, ctxo, lse, keep, x1, h2, mu2, rs2, f_pre, f = ctx.saved
        ctx.saved = None
        dy = dy.contiguous()
        C = x.shape[1]
        H = L.heads
        at = L.attention
        ln1, ln2, fc1, fc2 = L.layernorm_before, L.layernorm_after, L.mlp.fc1, L.mlp.fc2
        dfp = linear_bwd(dy, f, fc2.weight, fc2.bias, dt, act_bwd=ACT_GELU_ERF, aux=f_pre)
        dh2 = linear_bwd(dfp, h2, fc1.weight, fc1.bias, dt)
        dx1 = ops.layernorm_bwd(dh2, x1, ln2.weight.detach(), mu2, rs2, G(ln2.weight), G(ln2.bias), dres=dy)
        da = dx1 if keep is None else ops.rowscale_add(dx1, keep, Limg)
        dctx = linear_bwd(da, ctxo, at.o_proj.weight, at.o_proj.bias, dt)
        dqkv = torch.empty_like(qkv)
        tab = at.relative_position_bias.relative_position_bias_table
        ops.window_attn_bwd(qkv, C, H, ws, nW, scale, tab.detach(), labels, ctxo, dctx, lse, dqkv, G(tab))
        dh1 = linear_bwd(dqkv, h1, None, None, dt, fused=(at.qkv_w, at.qkv_b))
        dx = ops.layernorm_bwd(dh1, x, ln1.weight.detach(), mu1, rs1, G(ln1.weight), G(ln1.bias), dres=dx1)
        return dx, None, None, None, None, None, None


class _MergeFn(torch.autograd.Function):
    """SwinPatchMerging.forward (modeling_swin.py:309-326): 2x2 gather -> LN(4C) -> Linear(4C->2C)."""

    @staticmethod
    def forward(ctx, x, anchor, ds, idx, inv):
        dt = getattr(ds, "_capk_dtype", torch.bfloat16)
        C = x.shape[1]
        R4 = idx.numel() // 4
        g = _gather(x, idx, idx.numel()).view(R4, 4 * C)
        h, mu, rs = ops.layernorm_fwd(g, ds.norm.weight.detach(), ds.norm.bias.detach(), ds.norm.eps)
        y = ops.linear(h, W(ds.reduction.weight, dt))
        ctx.ds, ctx.inv, ctx.dt = ds, inv, dt
        ctx.saved = (g, h, mu, rs)
        return y

    @staticmethod
    def backward(ctx, dy):
        ds, dt = ctx.ds, ctx.dt
        g, h, mu, rs = ctx.saved
        ctx.saved = None
        dh = linear_bwd(dy.contiguous(), h, ds.reduction.weight, None, dt)
        dg = ops.layernorm_bwd(dh, g, ds.norm.weight.detach(), mu, rs, G(ds.norm.weight), G(ds.norm.bias))
        C = g.shape[1] // 4
        dx = _gather(dg.view(-1, C), ctx.inv, ctx.inv.numel())
        return dx, None, None, None, None


class SwinHeadFn(torch.autograd.Function):
    """SwinModel.layernorm (modeling_swin.py:876) -> SwinEncoder.proj (encoders.py:153-158,
    Linear or Identity) -> features.mean(dim=1) (encoders.py:172)."""

    @staticmethod
    def forward(ctx, x, anchor, m, proj, B, Limg):
        ctx.set_materialize_grads(False)
        dt = m.cdtype
        ln = m.layernorm
        seq, mu, rs = ops.layernorm_fwd(x, ln.weight.detach(), ln.bias.detach(), ln.eps)
        feats = seq if proj is None else ops.linear(seq, W(proj.weight, dt), proj.bias.detach())
        D = feats.shape[1]
        pooled = ops.avgpool_fwd(feats, B, Limg, 1, D, 1, 1)
        ctx.m, ctx.proj, ctx.B, ctx.Limg = m, proj, B, Limg
        ctx.saved = (x, mu, rs, seq)
        return feats, pooled

    @staticmethod
    def backward(ctx, dfeats, dpooled):
        m, proj, B, Limg = ctx.m, ctx.proj, ctx.B, ctx.Limg
        dt = m.cdtype
        x, mu, rs, seq = ctx.saved
        ctx.saved = None
        D = proj.weight.shape[0] if proj is not None else seq.shape[1]
        if dfeats is None:
            dfeats = torch.zeros(B * Limg, D, dtype=seq.dtype, device=seq.device)
        else:
            dfeats = dfeats.contiguous().clone() if dpooled is not None else dfeats.contiguous()
        if dpooled is not None:
            ops.avgpool_bwd(dpooled.contiguous(), B, Limg, 1, D, 1, 1, dx=dfeats, beta=1.0)
        dseq = dfeats if proj is None else linear_bwd(dfeats, seq, proj.weight, proj.bias, dt)
        ln = m.layernorm
        dx = ops.layernorm_bwd(dseq, x, ln.weight.detach(), mu, rs, G(ln.weight), G(ln.bias))
        return dx, None, None, None, None, None
