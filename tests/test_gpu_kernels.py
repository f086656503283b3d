"""Kernel-level parity: every libcapk kernel vs a plain PyTorch fp32 reference of the
same op (computed on the bf16-rounded inputs for the bf16 path).  GPU only."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")


@pytest.fixture(scope="module")
def ops():
    from capk import ops as _ops
    return _ops


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


# ------------------------------------------------ weight transposes (round 6) ----
@cuda
def test_transpose_bf16_batch(ops):
    """capk_transpose_bf16_batch: bit-exact transposes of ragged shapes (partial 64 x 64 edge
    tiles), strided sources, and more than 64 matrices (two launches)."""
    g = torch.Generator(device="cuda").manual_seed(0)
    shapes = [(8, 8), (72, 136), (768, 2304), (2304, 768), (64, 64), (200, 520)] + [(16, 24)] * 70
    pairs = []
    for i, (r, c) in enumerate(shapes):
        base = torch.randn(r, c + (8 if i % 3 == 1 else 0), device="cuda", generator=g).bfloat16()
        src = base[:, :c]  # (every third one a strided view)
        pairs.append((src, torch.full((c, r), float("nan"), device="cuda", dtype=torch.bfloat16)))
    ops.transpose_bf16_batch(pairs)
    for src, dst in pairs:
        assert torch.equal(dst, src.t()), tuple(src.shape)


@cuda
@pytest.mark.parametrize("N,K", [(2304, 768), (768, 3072), (768, 768)])
def test_linear_dx_weight_copy(ops, N, K):
    """ops.WeightT: the dX product on the K-major weight copy matches the N-major operand
    (fp32 reference of the bf16 inputs), follows an in-place weight change once
    weights_changed() is signalled, and is refreshed by ops.adamw writing the bf16 shadow."""
    g = torch.Generator(device="cuda").manual_seed(1)
    M = 4096
    shadow = torch.zeros(N * K + 4096, device="cuda", dtype=torch.bfloat16)
    ops.WT.register(shadow)
    w = shadow[:N * K].view(N, K)
    w.copy_((torch.randn(N, K, device="cuda", generator=g) / math.sqrt(N)).bfloat16())
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    wt = ops.WT.get(w, M)  # the copy path is taken, with an exact transpose
    assert wt is not None and torch.equal(wt, w.t())
    out = ops.linear_dx(dy, w)
    ref = dy.float() @ w.float()
    assert _rel(out, ref) < 1e-2
    ops.WT.enabled = False
    try:
        out_n = ops.linear_dx(dy, w)
    finally:
        ops.WT.enabled = True
    assert _rel(out, out_n) < 1e-2
    w.neg_()
    ops.WT.weights_changed()
    assert torch.equal(ops.WT.get(w, M), w.t())
    assert _rel(ops.linear_dx(dy, w), -ref) < 1e-2
    # the optimizer path: AdamW rewriting the bf16 shadow invalidates the copies by itself
    master = w.float().reshape(-1).contiguous()
    grad = torch.randn(master.numel(), device="cuda", generator=g)
    m, v = torch.zeros_like(master), torch.zeros_like(master)
    ops.adamw(master, grad, m, v, shadow[:N * K], 1e-2, 0.0, 0.9, 0.999, 1e-8, 1)
    assert torch.equal(ops.WT.get(w, M), w.t())
    assert _rel(ops.linear_dx(dy, w), dy.float() @ w.float()) < 1e-2
    # the overlapped refresh (CapkAdamW.step): transposes on a side stream right after the
    # update, awaited by the next dX product; a second update joins them before rewriting
    ops.WT.overlap = True
    try:
        for _ in range(2):
            ops.adamw(master, grad, m, v, shadow[:N * K], 1e-2, 0.0, 0.9, 0.999, 1e-8, 2)
            ops.WT.refresh_async()
        assert ops.WT.pending
        assert torch.equal(ops.WT.get(w, M), w.t())
    finally:
        ops.WT.overlap = False
    # views outside a registered shadow keep the N-major operand
    assert ops.WT.get(w.clone(), M) is None


# ------------------------------------------------------------------ GEMM ----
@cuda
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(300, 256, 192), (128, 128, 64), (517, 384, 768)])
def test_linear_fwd_epilogues(ops, dtype, M, N, K):
    from capk._lib import ACT_GELU_ERF
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device="cuda", generator=g).to(dtype)
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).to(dtype)
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g).to(dtype)
    pre = torch.empty(M, N, device="cuda", dtype=dtype)
    y = ops.linear(x, w, b, residual=r, act=ACT_GELU_ERF, preact=pre)
    ref_pre = x.float() @ w.float().t() + b
    ref = F.gelu(ref_pre) + r.float()  # capk.h: C = dropout(act(pre)) + residual
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(pre, ref_pre) < tol
    assert _rel(y, ref) < tol


@cuda
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_linear_backward_layouts(ops, dtype):
    from capk._lib import ACT_GELU_ERF
    g = torch.Generator(device="cuda").manual_seed(1)
    M, N, K = 777, 384, 256
    dy = torch.randn(M, N, device="cuda", generator=g).to(dtype)
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(N)).to(dtype)
    x = torch.randn(M, K, device="cuda", generator=g).to(dtype)
    aux = torch.randn(M, K, device="cuda", generator=g).to(dtype)
    dx = ops.linear_dx(dy, w)
    assert _rel(dx, dy.float() @ w.float()) < (1e-5 if dtype == torch.float32 else 1e-2)
    # fused activation backward: dX * gelu'(aux)
    dxa = ops.linear_dx(dy, w, act_bwd=ACT_GELU_ERF, aux=aux)
    a = aux.float().requires_grad_(True)
    F.gelu(a).backward(dy.float() @ w.float())
    assert _rel(dxa, a.grad) < (1e-5 if dtype == torch.float32 else 1e-2)
    dw = torch.empty(N, K, device="cuda", dtype=torch.float32)
    ops.linear_dw(dy, x, dw)
    assert _rel(dw, dy.float().t() @ x.float()) < (1e-5 if dtype == torch.float32 else 5e-3)


@cuda
@pytest.mark.parametrize("cfg", [1, 7, 8, 9])
@pytest.mark.parametrize("M,N,K", [(1280, 768, 768), (300, 256, 192), (517, 384, 3072), (70, 3072, 768)])
def test_ring_configs_bf16(ops, cfg, M, N, K):
    """The 128x128 ring tiles (1: 2-deep, 7: 4-deep, one WG per CU), the 64x128 tile (8: two
    waves) and the 64x64 four-wave tile (9: gemm_s64_kernel, no split-K), forced in turn on K-major products with ragged M / N: bias + GELU (kept pre-act) +
    residual epilogue, and a plain product whose K split takes the slab reduce, vs the fp32
    product of the same bf16 values."""
    from capk._lib import ACT_GELU_ERF
    L = ops.lib()
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    try:
        ops.check(L.capk_gemm_force_config(cfg), "force_config")
        y = ops.linear(x, w, b, residual=r, act=ACT_GELU_ERF, preact=pre)
        assert L.capk_gemm_last_config() == cfg
        yp = ops.linear(x, w)
    finally:
        L.capk_gemm_force_config(-1)
    ref_pre = x.float() @ w.float().t() + b
    assert _rel(pre, ref_pre) < 1e-2
    assert _rel(y, F.gelu(ref_pre) + r.float()) < 1e-2
    assert _rel(yp, x.float() @ w.float().t()) < 1e-2


@cuda
@pytest.mark.parametrize("M,N,K", [(1280, 768, 768), (1280, 1536, 1536), (1280, 2304, 768), (1280, 3072, 768)])
def test_s64_ring_depths(ops, M, N, K):
    """The 64x64 decode tile (cfg 9) on one-round and multi-round grids (240 / 480 / 720 WGs: the
    3-deep ring; 960: the 2-deep ring) with the bias + GELU + residual epilogue, vs the fp32 product
    of the same bf16 values (the split-K slab route: test_product_ln_slabs_bit_identical)."""
    from capk._lib import ACT_GELU_ERF
    L = ops.lib()
    g = torch.Generator(device="cuda").manual_seed(19)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    try:
        ops.check(L.capk_gemm_force_config(9), "force_config")
        y = ops.linear(x, w, b, residual=r, act=ACT_GELU_ERF, preact=pre)
        assert L.capk_gemm_last_config() == 9
    finally:
        L.capk_gemm_force_config(-1)
    ref_pre = x.float() @ w.float().t() + b
    assert _rel(pre, ref_pre) < 1e-2
    assert _rel(y, F.gelu(ref_pre) + r.float()) < 1e-2


@cuda
def test_gemm_bf16_splitk_and_beta(ops):
    """dW-shaped GEMM with a long reduction (split-K slabs + reduce) and accumulate."""
    g = torch.Generator(device="cuda").manual_seed(2)
    M, N, K = 8192, 256, 384  # dy [M,N], x [M,K]: dW [N,K] reduces over M
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    dw = torch.randn(N, K, device="cuda", generator=g)
    dw0 = dw.clone()
    ops.linear_dw(dy, x, dw, accumulate=True)
    ref = dw0 + dy.float().t() @ x.float()
    assert _rel(dw, ref) < 5e-3


@cuda
def test_gemm_bf16_strided_rows_and_beta_output(ops):
    """A with row stride > K (CLS rows of a [B,N,D] buffer) and C written with ldc, beta=1."""
    g = torch.Generator(device="cuda").manual_seed(3)
    B, Ntok, D = 40, 5, 128
    seq = torch.randn(B * Ntok, D, device="cuda", generator=g).bfloat16()
    cls = seq.view(B, Ntok, D)[:, 0]
    w = (torch.randn(D, D, device="cuda", generator=g) / math.sqrt(D)).bfloat16()
    y = ops.linear(cls, w)
    assert _rel(y, cls.float() @ w.float().t()) < 1e-2
    out = torch.randn(B * Ntok, D, device="cuda", generator=g).bfloat16()
    o0 = out.clone()
    tgt = out.view(B, Ntok, D)[:, 0]
    ops.linear_dx(y, w, out=tgt, beta=1.0)
    ref = o0.view(B, Ntok, D)[:, 0].float() + y.float() @ w.float()
    assert _rel(out.view(B, Ntok, D)[:, 0], ref) < 1e-2
    assert torch.equal(out.view(B, Ntok, D)[:, 1:], o0.view(B, Ntok, D)[:, 1:])


# ------------------------------------------------------------- LayerNorm ----
@cuda
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols,eps", [(768, 1e-12), (1536, 1e-5), (32, 1e-5), (2048, 1e-5)])
def test_layernorm(ops, dtype, cols, eps):
    g = torch.Generator(device="cuda").manual_seed(4)
    rows = 1000
    x = (torch.randn(rows, cols, device="cuda", generator=g) * 3 + 1).to(dtype)
    w = torch.randn(cols, device="cuda", generator=g)
    b = torch.randn(cols, device="cuda", generator=g)
    dy = torch.randn(rows, cols, device="cuda", generator=g).to(dtype)
    dres = torch.randn(rows, cols, device="cuda", generator=g).to(dtype)
    y, mu, rs = ops.layernorm_fwd(x, w, b, eps)
    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = F.layer_norm(xr, (cols,), wr, br, eps)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(y, yr) < tol
    yr.backward(dy.float())
    dw = torch.empty(cols, device="cuda")
    db = torch.empty(cols, device="cuda")
    dsum = torch.empty(cols, device="cuda")
    dx = ops.layernorm_bwd(dy, x, w, mu, rs, dw, db, dres=dres, dsum=dsum)
    assert _rel(dx, xr.grad + dres.float()) < tol
    # fused bias gradient: column sums of dx, accumulated in fp32 before dx is rounded to the
    # storage dtype -> compared with the fp32 reference's column sums
    assert _rel(dsum, (xr.grad + dres.float()).sum(0)) < (1e-5 if dtype == torch.float32 else 5e-3)
    dx2 = ops.layernorm_bwd(dy, x, w, mu, rs, dw, db, dres=dres)  # without dsum: same dx
    assert torch.equal(dx2, dx)
    assert _rel(dw, wr.grad) < (1e-5 if dtype == torch.float32 else 5e-3)
    assert _rel(db, br.grad) < (1e-5 if dtype == torch.float32 else 5e-3)


# ------------------------------------------------------------- attention ----
def _attn_ref(q, k, v, scale, causal, key_pad):
    s = torch.einsum("bhqd,bhkd->bhqk", q, k) * scale
    if causal:
        Nq, Nk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Nq, Nk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    if key_pad is not None:
        s = s.masked_fill(key_pad[:, None, None, :], float("-inf"))
    return torch.einsum("bhqk,bhkd->bhqd", torch.softmax(s, -1), v)


@cuda
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", ["vit", "dec_self", "dec_cross_gap", "clip", "vit_stream", "pad_stream",
                                  "causal_stream", "clip_stream_gap"])
def test_attention_fwd_bwd(ops, dtype, case):
    """Per-(batch, head) kernels at the config shapes and at >= 1024 (batch, head) pairs
    (*_stream; clip_stream_gap: a gap row between images, Nq = 50)."""
    from capk.ops import HeadView
    g = torch.Generator(device="cuda").manual_seed(5)
    if case == "vit_stream":
        B, H, Nq, Nk, hd, causal, gap = 96, 12, 197, 197, 64, False, 0
    elif case == "pad_stream":
        B, H, Nq, Nk, hd, causal, gap = 128, 8, 50, 50, 64, False, 1
    elif case == "causal_stream":
        B, H, Nq, Nk, hd, causal, gap = 128, 8, 40, 40, 64, True, 0
    elif case == "clip_stream_gap":
        B, H, Nq, Nk, hd, causal, gap = 90, 12, 50, 50, 64, False, 1
    elif case == "vit":
        B, H, Nq, Nk, hd, causal, gap = 3, 4, 197, 197, 64, False, 0
    elif case == "dec_self":
        B, H, Nq, Nk, hd, causal, gap = 4, 8, 20, 20, 96, True, 0
    elif case == "dec_cross_gap":
        B, H, Nq, Nk, hd, causal, gap = 3, 8, 20, 196, 96, False, 1
    else:
        B, H, Nq, Nk, hd, causal, gap = 5, 12, 50, 50, 64, False, 0
    D = H * hd
    q = torch.randn(B * Nq, D, device="cuda", generator=g).to(dtype)
    kvrows = (B - 1) * (Nk + gap) + Nk
    kv = torch.randn(kvrows, 2 * D, device="cuda", generator=g).to(dtype)
    do = torch.randn(B * Nq, D, device="cuda", generator=g).to(dtype)
    key_pad = None
    if case in ("dec_self", "pad_stream"):
        key_pad = torch.zeros(B, Nk, dtype=torch.bool, device="cuda")
        key_pad[1, 15:] = True
        key_pad[3, 19] = True
        if case == "pad_stream":
            key_pad[7:, 33:] = True
    o = torch.empty(B * Nq, D, device="cuda", dtype=dtype)
    qv = HeadView(q, 0, Nq * D, D)
    kview = HeadView(kv, 0, (Nk + gap) * 2 * D, 2 * D)
    vview = HeadView(kv, D, (Nk + gap) * 2 * D, 2 * D)
    ov = HeadView(o, 0, Nq * D, D)
    scale = 1.0 / math.sqrt(hd)
    lse, kp = ops.attention_fwd(qv, kview, vview, ov, B, H, Nq, Nk, hd, scale, causal=causal, key_pad=key_pad)

    def heads_of(t, rows_per_b, n, col0):
        t = t.float()
        out = torch.stack([t[b * rows_per_b:b * rows_per_b + n, col0:col0 + D] for b in range(B)])
        return out.view(B, n, H, hd).transpose(1, 2).contiguous()

    qr = heads_of(q, Nq, Nq, 0).requires_grad_(True)
    kr = heads_of(kv, Nk + gap, Nk, 0).requires_grad_(True)
    vr = heads_of(kv, Nk + gap, Nk, D).requires_grad_(True)
    ref = _attn_ref(qr, kr, vr, scale, causal, key_pad)
    got = o.float().view(B, Nq, H, hd).transpose(1, 2)
    tol = 1e-5 if dtype == torch.float32 else 1.5e-2
    assert _rel(got, ref) < tol
    ref.backward(do.float().view(B, Nq, H, hd).transpose(1, 2))
    dq = torch.empty_like(q)
    dkv = torch.zeros_like(kv)
    ops.attention_bwd(qv, kview, vview, ov, HeadView(do, 0, Nq * D, D), lse, HeadView(dq, 0, Nq * D, D),
                      HeadView(dkv, 0, (Nk + gap) * 2 * D, 2 * D), HeadView(dkv, D, (Nk + gap) * 2 * D, 2 * D),
                      B, H, Nq, Nk, hd, scale, causal=causal, key_pad_u8=kp)
    tolb = 1e-4 if dtype == torch.float32 else 3e-2
    assert _rel(dq.float().view(B, Nq, H, hd).transpose(1, 2), qr.grad) < tolb
    assert _rel(heads_of(dkv, Nk + gap, Nk, 0), kr.grad) < tolb
    assert _rel(heads_of(dkv, Nk + gap, Nk, D), vr.grad) < tolb
    if gap:
        gap_rows = torch.stack([dkv[b * (Nk + gap) + Nk] for b in range(B - 1)])
        assert float(gap_rows.abs().max()) == 0.0


@cuda
@pytest.mark.parametrize("case", ["self_step", "cross_beams", "pad", "hd64_q8", "gpt2_step", "cross_one",
                                  "cross_pad", "cross_hd128_q16"])
def test_attention_decode_bf16(ops, case):
    """Small-Nq decode path (attn_decode2_bf16, chosen automatically for Nq <= 8): KV-cache
    self-attention (one query, strided cache rows) and beam cross-attention (k beam
    queries of one image against shared memory keys with a CLS gap row)."""
    from capk.ops import HeadView
    g = torch.Generator(device="cuda").manual_seed(11)
    pad = None
    if case == "self_step":
        B, H, Nq, Nk, hd, gap, Lm = 40, 8, 1, 13, 96, 0, 20
    elif case == "cross_beams":
        B, H, Nq, Nk, hd, gap, Lm = 6, 8, 5, 196, 96, 1, 0
    elif case == "pad":
        B, H, Nq, Nk, hd, gap, Lm = 4, 4, 3, 37, 32, 0, 0
        pad = torch.zeros(B, Nk, dtype=torch.bool, device="cuda")
        pad[1, 30:] = True
        pad[2, 0] = True
    elif case == "gpt2_step":  # GPT-2 KV cache: 10 prefix slots + 19 tokens, hd 64
        B, H, Nq, Nk, hd, gap, Lm = 48, 12, 1, 29, 64, 0, 30
    elif case == "cross_one":  # greedy cross step: one query against 196 memory keys (7 waves merged)
        B, H, Nq, Nk, hd, gap, Lm = 7, 8, 1, 196, 96, 1, 0
    elif case == "cross_pad":  # MFMA beam-cross kernel (attn_xdec_bf16) with padded memory keys
        B, H, Nq, Nk, hd, gap, Lm = 4, 8, 5, 150, 96, 0, 0
        pad = torch.zeros(B, Nk, dtype=torch.bool, device="cuda")
        pad[1, 70:] = True   # a wave's whole key range padded
        pad[3, ::3] = True
    elif case == "cross_hd128_q16":  # 16 queries (one full MFMA query tile), hd 128
        B, H, Nq, Nk, hd, gap, Lm = 3, 4, 16, 200, 128, 0, 0
    else:
        B, H, Nq, Nk, hd, gap, Lm = 5, 12, 8, 256, 64, 0, 0
    D = H * hd
    dtype = torch.bfloat16
    if Lm:  # [B, Lm, 3D] cache; query = row Nk-1's q slot
        cache = torch.randn(B, Lm, 3 * D, device="cuda", generator=g).to(dtype)
        qv = HeadView(cache, (Nk - 1) * 3 * D, Lm * 3 * D, 3 * D)
        kview = HeadView(cache, D, Lm * 3 * D, 3 * D)
        vview = HeadView(cache, 2 * D, Lm * 3 * D, 3 * D)
        qr = cache[:, Nk - 1:Nk, :D].float()
        kr, vr = cache[:, :Nk, D:2 * D].float(), cache[:, :Nk, 2 * D:].float()
    else:
        q = torch.randn(B * Nq, D, device="cuda", generator=g).to(dtype)
        kv = torch.randn((B - 1) * (Nk + gap) + Nk, 2 * D, device="cuda", generator=g).to(dtype)
        qv = HeadView(q, 0, Nq * D, D)
        kview = HeadView(kv, 0, (Nk + gap) * 2 * D, 2 * D)
        vview = HeadView(kv, D, (Nk + gap) * 2 * D, 2 * D)
        qr = q.float().view(B, Nq, D)
        kr = torch.stack([kv[b * (Nk + gap):b * (Nk + gap) + Nk, :D] for b in range(B)]).float()
        vr = torch.stack([kv[b * (Nk + gap):b * (Nk + gap) + Nk, D:] for b in range(B)]).float()
    o = torch.empty(B * Nq, D, device="cuda", dtype=dtype)
    scale = 1.0 / math.sqrt(hd)
    lse, _ = ops.attention_fwd(qv, kview, vview, HeadView(o, 0, Nq * D, D), B, H, Nq, Nk, hd, scale, key_pad=pad)
    sp = lambda t, n: t.reshape(B, n, H, hd).transpose(1, 2)  # noqa: E731
    ref = _attn_ref(sp(qr, Nq), sp(kr, Nk), sp(vr, Nk), scale, False, pad)
    got = o.float().view(B, Nq, H, hd).transpose(1, 2)
    assert _rel(got, ref) < 1e-2
    s = torch.einsum("bhqd,bhkd->bhqk", sp(qr, Nq), sp(kr, Nk)) * scale
    if pad is not None:
        s = s.masked_fill(pad[:, None, None, :], float("-inf"))
    torch.testing.assert_close(lse, torch.logsumexp(s, -1), rtol=1e-4, atol=1e-4)


# ------------------------------------------------------ CE / embeddings -----
@cuda
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_shifted_ce(ops, dtype):
    g = torch.Generator(device="cuda").manual_seed(6)
    B, T, V = 6, 9, 50257
    Vp = (V + 63) // 64 * 64
    logits = torch.randn(B * T, Vp, device="cuda", generator=g).to(dtype)
    tg = torch.randint(0, V, (B, T), device="cuda", generator=g)
    pad = V - 1
    tg[2, 4:] = pad
    loss = ops.shifted_ce(logits, tg, B, T, V, pad)
    lr = logits.float()[:, :V].view(B, T, V).requires_grad_(True)
    ref = F.cross_entropy(lr[:, :-1].reshape(-1, V), tg[:, 1:].reshape(-1), ignore_index=pad)
    assert abs(float(loss[0]) - float(ref)) < 1e-4 * max(1.0, abs(float(ref)))
    ref.backward()
    dl = torch.empty_like(logits)
    gs = torch.tensor([0.5], device="cuda")
    ops.shifted_ce(logits, tg, B, T, V, pad, want_loss=False, dlogits=dl, grad_scale=gs)
    assert _rel(dl[:, :V].view(B, T, V), 0.5 * lr.grad) < (1e-5 if dtype == torch.float32 else 1e-2)
    assert float(dl[:, V:].float().abs().max()) == 0.0


@cuda
def test_embedding_fwd_bwd(ops):
    g = torch.Generator(device="cuda").manual_seed(7)
    B, T, D, V = 4, 7, 64, 100
    ids = torch.randint(0, V, (B, T), device="cuda", generator=g)
    ids[0, 3] = 5
    table = torch.randn(V, D, device="cuda", generator=g)
    pos = torch.randn(50, D, device="cuda", generator=g)
    out = ops.embedding_fwd(ids, table, pos, 0, torch.float32)
    assert torch.allclose(out.view(B, T, D), table[ids] + pos[:T][None], atol=1e-6)
    dout = torch.randn(B * T, D, device="cuda", generator=g)
    dt = torch.zeros(V, D, device="cuda")
    dp = torch.zeros(50, D, device="cuda")
    ops.embedding_bwd(ids, dout, 5, dt, dp, 0)
    ref_t = torch.zeros(V, D, device="cuda").index_add_(0, ids.reshape(-1), dout)
    ref_t[5] = 0
    assert torch.allclose(dt, ref_t, atol=1e-5)
    assert torch.allclose(dp[:T], dout.view(B, T, D).sum(0), atol=1e-5)


@cuda
def test_adamw_matches_oracle(ops):
    from oracle import train as otrain
    g = torch.Generator(device="cuda").manual_seed(8)
    n = 1000003
    p = torch.randn(n, device="cuda", generator=g)
    gr = torch.randn(n, device="cuda", generator=g)
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    sh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    pc, mc, vc = p.cpu(), m.cpu(), v.cpu()
    for step in (1, 2, 3):
        ops.adamw(p, gr, m, v, sh, 1e-3, 0.01, 0.9, 0.999, 1e-8, step)
        otrain.adamw_step(pc, gr.cpu(), mc, vc, step, 1e-3, 0.01)
    torch.testing.assert_close(p.cpu(), pc, rtol=1e-6, atol=1e-7)
    assert torch.equal(sh, p.bfloat16())


@cuda
def test_patchify_assemble(ops):
    g = torch.Generator(device="cuda").manual_seed(9)
    B, C, Hh, Ww, P, D = 3, 3, 32, 32, 8, 64
    img = torch.randn(B, C, Hh, Ww, device="cuda", generator=g)
    pt = ops.patchify(img, P, torch.float32)
    ref = F.unfold(img, P, stride=P).transpose(1, 2).reshape(-1, C * P * P)
    assert torch.equal(pt, ref)
    Np = (Hh // P) * (Ww // P)
    pe = torch.randn(B * Np, D, device="cuda", generator=g)
    cls = torch.randn(D, device="cuda", generator=g)
    pos = torch.randn(Np + 1, D, device="cuda", generator=g)
    x = ops.vit_assemble(pe, cls, pos, B, Np, D).view(B, Np + 1, D)
    ref = torch.cat([cls.expand(B, 1, D), pe.view(B, Np, D)], 1) + pos
    assert torch.allclose(x, ref)
    dx = torch.randn(B * (Np + 1), D, device="cuda", generator=g)
    dcls = torch.empty(D, device="cuda")
    dpos = torch.empty(Np + 1, D, device="cuda")
    dpatch = ops.vit_assemble_bwd(dx, B, Np, D, dcls, dpos)
    assert torch.equal(dpatch.view(B, Np, D), dx.view(B, Np + 1, D)[:, 1:])
    assert torch.allclose(dpos, dx.view(B, Np + 1, D).sum(0), atol=1e-5)
    assert torch.allclose(dcls, dx.view(B, Np + 1, D)[:, 0].sum(0), atol=1e-5)


# ---------------------------------------------------------------- dropout ---
@cuda
def test_dropout_mask_statistics_and_gemm_epilogue(ops):
    from capk._lib import ACT_GELU_ERF
    m = ops.dropout_mask(1 << 20, 0.1, 1234).float()
    assert abs(float(m.mean()) - 0.9) < 3e-3
    g = torch.Generator(device="cuda").manual_seed(11)
    M, N, K = 300, 256, 128
    x = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g)
    mk = ops.dropout_mask(M * N, 0.25, 77).view(M, N).float() / 0.75
    for dt, tol in ((torch.float32, 1e-5), (torch.bfloat16, 1e-2)):
        pre = torch.empty(M, N, device="cuda", dtype=dt)
        y = ops.linear(x.to(dt), w.to(dt), b, residual=r.to(dt), act=ACT_GELU_ERF, preact=pre, drop=(0.25, 77))
        ref = F.gelu(x.to(dt).float() @ w.to(dt).float().t() + b) * mk + r.to(dt).float()
        assert _rel(y, ref) < tol


@cuda
def test_attention_dropout_fwd_bwd(ops):
    from capk.ops import HeadView
    g = torch.Generator(device="cuda").manual_seed(12)
    B, H, Nq, Nk, hd, p, seed = 3, 4, 20, 37, 32, 0.2, 4242
    D = H * hd
    for dt, tol, tolb in ((torch.float32, 1e-5, 1e-4), (torch.bfloat16, 1.5e-2, 3e-2)):
        q = torch.randn(B * Nq, D, device="cuda", generator=g).to(dt)
        kv = torch.randn(B * Nk, 2 * D, device="cuda", generator=g).to(dt)
        do = torch.randn(B * Nq, D, device="cuda", generator=g).to(dt)
        o = torch.empty(B * Nq, D, device="cuda", dtype=dt)
        Q, K_, V_, O = HeadView(q, 0, Nq * D, D), HeadView(kv, 0, Nk * 2 * D, 2 * D), HeadView(kv, D, Nk * 2 * D, 2 * D), HeadView(o, 0, Nq * D, D)
        sc = 1 / math.sqrt(hd)
        lse, _ = ops.attention_fwd(Q, K_, V_, O, B, H, Nq, Nk, hd, sc, drop=(p, seed))
        mk = ops.dropout_mask(B * H * Nq * Nk, p, seed).view(B, H, Nq, Nk).float() / (1 - p)
        qr = q.float().view(B, Nq, H, hd).transpose(1, 2).requires_grad_(True)
        kr = kv.float()[:, :D].reshape(B, Nk, H, hd).transpose(1, 2).detach().requires_grad_(True)
        vr = kv.float()[:, D:].reshape(B, Nk, H, hd).transpose(1, 2).detach().requires_grad_(True)
        ref = (torch.softmax(qr @ kr.transpose(-1, -2) * sc, -1) * mk) @ vr
        assert _rel(o.float().view(B, Nq, H, hd).transpose(1, 2), ref) < tol
        ref.backward(do.float().view(B, Nq, H, hd).transpose(1, 2))
        dq, dkv = torch.empty_like(q), torch.empty_like(kv)
        ops.attention_bwd(Q, K_, V_, O, HeadView(do, 0, Nq * D, D), lse, HeadView(dq, 0, Nq * D, D),
                          HeadView(dkv, 0, Nk * 2 * D, 2 * D), HeadView(dkv, D, Nk * 2 * D, 2 * D), B, H, Nq, Nk, hd,
                          sc, drop=(p, seed))
        assert _rel(dq.float().view(B, Nq, H, hd).transpose(1, 2), qr.grad) < tolb
        assert _rel(dkv.float()[:, :D].reshape(B, Nk, H, hd).transpose(1, 2), kr.grad) < tolb
        assert _rel(dkv.float()[:, D:].reshape(B, Nk, H, hd).transpose(1, 2), vr.grad) < tolb


@cuda
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("deriv", [False, True])
def test_act_bwd_colsum(ops, dtype, deriv):
    """capk_act_bwd_colsum: c <- c * GELU'(aux) (or * aux with CAPK_ACT_DERIV) in place, db = colsum
    (the FC1 bias gradient fused into the FC2-dX activation pass), vs torch fp32."""
    from capk._lib import ACT_DERIV, ACT_GELU_ERF
    g = torch.Generator(device="cuda").manual_seed(9)
    M, N = 1037, 3072  # M not a multiple of the 256-row split or of the 8-row unroll
    c = torch.randn(M, N, device="cuda", generator=g).to(dtype)
    aux = torch.randn(M, N, device="cuda", generator=g).to(dtype)
    xr = aux.float().requires_grad_(True)
    if deriv:
        ref = c.float() * aux.float()
    else:
        F.gelu(xr).backward(c.float())
        ref = xr.grad
    db = torch.full((N,), 7.0, device="cuda")
    out = ops.act_bwd_colsum(c, aux, ACT_GELU_ERF | (ACT_DERIV if deriv else 0), db)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert out.data_ptr() == c.data_ptr()
    assert _rel(c, ref) < tol, _rel(c, ref)
    assert _rel(db, ref.sum(0)) < (1e-5 if dtype == torch.float32 else 5e-3), _rel(db, ref.sum(0))
    db2 = db.clone()
    ops.act_bwd_colsum(c.clone(), aux, ACT_GELU_ERF | (ACT_DERIV if deriv else 0), db2, accumulate=True)
    assert db2.shape == db.shape and bool(torch.isfinite(db2).all())


@cuda
@pytest.mark.parametrize("case", ["dec_cross_drop", "qformer_cross", "cross_q16_pad"])
def test_cross_attention_xdec_train(ops, case):
    """Short query blocks against memory keys on the MFMA xdec kernel (chosen for 2 <= Nq <= 32,
    64 < Nk <= 256, hd 64 / 96 / 128): the training decoder's cross-attention (Nq = 20 caption
    positions, Nk = 196 memory keys, hd 96) with probability dropout p = 0.1 -- the mask is
    materialised by capk_dropout_mask at index ((b*H + h)*Nq + q)*Nk + key, as attn_bwd
    recomputes it -- the QFormer's 32 queries (two query tiles, hd 64), and 16 queries with a
    key-padding mask; forward (O, and the lse through the backward) and the backward that
    consumes it, bf16 vs an fp32 reference on the bf16 inputs."""
    from capk.ops import HeadView
    g = torch.Generator(device="cuda").manual_seed(17)
    p, seed = 0.0, 0
    key_pad = None
    if case == "dec_cross_drop":
        B, H, Nq, Nk, hd = 24, 8, 20, 196, 96
        p, seed = 0.1, 4242
    elif case == "qformer_cross":
        B, H, Nq, Nk, hd = 10, 12, 32, 196, 64
    else:
        B, H, Nq, Nk, hd = 6, 4, 16, 150, 128
        key_pad = torch.zeros(B, Nk, dtype=torch.bool, device="cuda")
        key_pad[1, 100:] = True
        key_pad[4, 7] = True
    D = H * hd
    dt = torch.bfloat16
    q = torch.randn(B * Nq, D, device="cuda", generator=g).to(dt)
    kv = torch.randn(B * Nk, 2 * D, device="cuda", generator=g).to(dt)
    do = torch.randn(B * Nq, D, device="cuda", generator=g).to(dt)
    o = torch.empty(B * Nq, D, device="cuda", dtype=dt)
    qv, ov = HeadView(q, 0, Nq * D, D), HeadView(o, 0, Nq * D, D)
    kview, vview = HeadView(kv, 0, Nk * 2 * D, 2 * D), HeadView(kv, D, Nk * 2 * D, 2 * D)
    scale = 1.0 / math.sqrt(hd)
    lse, kp = ops.attention_fwd(qv, kview, vview, ov, B, H, Nq, Nk, hd, scale, key_pad=key_pad, drop=(p, seed))
    qr = q.float().view(B, Nq, H, hd).transpose(1, 2).contiguous().requires_grad_(True)
    kr = kv[:, :D].float().reshape(B, Nk, H, hd).transpose(1, 2).contiguous().requires_grad_(True)
    vr = kv[:, D:].float().reshape(B, Nk, H, hd).transpose(1, 2).contiguous().requires_grad_(True)
    s = torch.einsum("bhqd,bhkd->bhqk", qr, kr) * scale
    if key_pad is not None:
        s = s.masked_fill(key_pad[:, None, None, :], float("-inf"))
    a = torch.softmax(s, -1)
    if p > 0:
        a = a * (ops.dropout_mask(B * H * Nq * Nk, p, seed).view(B, H, Nq, Nk).float() / (1 - p))
    ref = torch.einsum("bhqk,bhkd->bhqd", a, vr)
    got = o.float().view(B, Nq, H, hd).transpose(1, 2)
    assert _rel(got, ref) < 1.5e-2
    ref_lse = torch.logsumexp(s, -1)
    assert _rel(lse, ref_lse) < 1e-3
    ref.backward(do.float().view(B, Nq, H, hd).transpose(1, 2))
    dq = torch.empty_like(q)
    dkv = torch.zeros_like(kv)
    ops.attention_bwd(qv, kview, vview, ov, HeadView(do, 0, Nq * D, D), lse, HeadView(dq, 0, Nq * D, D),
                      HeadView(dkv, 0, Nk * 2 * D, 2 * D), HeadView(dkv, D, Nk * 2 * D, 2 * D),
                      B, H, Nq, Nk, hd, scale, key_pad_u8=kp, drop=(p, seed))
    assert _rel(dq.float().view(B, Nq, H, hd).transpose(1, 2), qr.grad) < 3e-2
    assert _rel(dkv[:, :D].float().reshape(B, Nk, H, hd).transpose(1, 2), kr.grad) < 3e-2
    assert _rel(dkv[:, D:].float().reshape(B, Nk, H, hd).transpose(1, 2), vr.grad) < 3e-2


@cuda
@pytest.mark.parametrize("case", ["dec_self_drop", "qformer_self", "gpt2_prefix"])
def test_short_attention_train(ops, case):
    """Short sequences on the one-wave-per-(batch, head) kernels (chosen for 8 < Nq <= 32,
    Nk <= 32): the training decoder's causal self-attention (T = 20, hd 96) with the caption
    key-padding mask and probability dropout p = 0.1 (mask materialised by capk_dropout_mask
    at ((b*H + h)*Nq + q)*Nk + key, as the backward recomputes it), the QFormer's 32 queries
    (hd 64, no mask), and a causal 20-query block over 30 keys (a 10-slot prefix, bottom-right
    aligned); forward, lse and backward, bf16 vs an fp32 reference on the bf16 inputs."""
    from capk.ops import HeadView
    g = torch.Generator(device="cuda").manual_seed(23)
    p, seed, causal, key_pad = 0.0, 0, False, None
    if case == "dec_self_drop":
        B, H, Nq, Nk, hd = 40, 8, 20, 20, 96
        p, seed, causal = 0.1, 777, True
        key_pad = torch.zeros(B, Nk, dtype=torch.bool, device="cuda")
        key_pad[1, 12:] = True
        key_pad[5, 19] = True
    elif case == "qformer_self":
        B, H, Nq, Nk, hd = 12, 12, 32, 32, 64
    else:
        B, H, Nq, Nk, hd = 9, 12, 20, 30, 64
        causal = True
    D = H * hd
    dt = torch.bfloat16
    q = torch.randn(B * Nq, D, device="cuda", generator=g).to(dt)
    kv = torch.randn(B * Nk, 2 * D, device="cuda", generator=g).to(dt)
    do = torch.randn(B * Nq, D, device="cuda", generator=g).to(dt)
    o = torch.empty(B * Nq, D, device="cuda", dtype=dt)
    qv, ov = HeadView(q, 0, Nq * D, D), HeadView(o, 0, Nq * D, D)
    kview, vview = HeadView(kv, 0, Nk * 2 * D, 2 * D), HeadView(kv, D, Nk * 2 * D, 2 * D)
    scale = 1.0 / math.sqrt(hd)
    lse, kp = ops.attention_fwd(qv, kview, vview, ov, B, H, Nq, Nk, hd, scale, causal=causal, key_pad=key_pad,
                                drop=(p, seed))
    qr = q.float().view(B, Nq, H, hd).transpose(1, 2).contiguous().requires_grad_(True)
    kr = kv[:, :D].float().reshape(B, Nk, H, hd).transpose(1, 2).contiguous().requires_grad_(True)
    vr = kv[:, D:].float().reshape(B, Nk, H, hd).transpose(1, 2).contiguous().requires_grad_(True)
    s = torch.einsum("bhqd,bhkd->bhqk", qr, kr) * scale
    if causal:  # bottom-right aligned: key j visible to query i when j <= i + Nk - Nq
        s = s.masked_fill(torch.ones(Nq, Nk, dtype=torch.bool, device="cuda").triu(1 + Nk - Nq), float("-inf"))
    if key_pad is not None:
        s = s.masked_fill(key_pad[:, None, None, :], float("-inf"))
    a = torch.softmax(s, -1)
    if p > 0:
        a = a * (ops.dropout_mask(B * H * Nq * Nk, p, seed).view(B, H, Nq, Nk).float() / (1 - p))
    ref = torch.einsum("bhqk,bhkd->bhqd", a, vr)
    got = o.float().view(B, Nq, H, hd).transpose(1, 2)
    assert _rel(got, ref) < 1.5e-2
    assert _rel(lse, torch.logsumexp(s, -1)) < 1e-3
    ref.backward(do.float().view(B, Nq, H, hd).transpose(1, 2))
    dq = torch.empty_like(q)
    dkv = torch.zeros_like(kv)
    ops.attention_bwd(qv, kview, vview, ov, HeadView(do, 0, Nq * D, D), lse, HeadView(dq, 0, Nq * D, D),
                      HeadView(dkv, 0, Nk * 2 * D, 2 * D), HeadView(dkv, D, Nk * 2 * D, 2 * D),
                      B, H, Nq, Nk, hd, scale, causal=causal, key_pad_u8=kp, drop=(p, seed))
    assert _rel(dq.float().view(B, Nq, H, hd).transpose(1, 2), qr.grad) < 3e-2
    assert _rel(dkv[:, :D].float().reshape(B, Nk, H, hd).transpose(1, 2), kr.grad) < 3e-2
    assert _rel(dkv[:, D:].float().reshape(B, Nk, H, hd).transpose(1, 2), vr.grad) < 3e-2


@cuda
@pytest.mark.parametrize("case", ["vit", "vit_split", "mask_drop", "mask_drop_split", "hd128", "short", "fp32"])
def test_attention_bwd_qkv_bias(ops, case):
    """capk_attention_bwd_bias: the backward plus the fused QKV bias gradient dbias = [colsum dQ |
    colsum dK | colsum dV] over the B*N tokens (the ViT query / key / value bias gradients,
    modeling_vit.py:205-216).  ViT self-attention (N = 197, hd 64) rides on the fused single-pass
    kernel (round 6: column sums of the bf16 values it stores, equal to the column sums of its own
    gradients to fp32 rounding, gradients bit-identical to the plain backward) or, *_split, on
    the split kernels (dQ sums from sum_q dS x K in the dK/dV kernel, dK / dV sums from per-query
    dS / P~ sums x Q / dO in the dQ kernel); key padding + dropout, hd 128, and the short / fp32
    routes (separate column sums) are checked against the fp32 autograd reference and against
    the column sums of the kernel's own gradients; accumulate adds."""
    from capk.ops import HeadView
    L = ops.lib()
    g = torch.Generator(device="cuda").manual_seed(31)
    p, seed, key_pad, dt = 0.0, 0, None, torch.bfloat16
    split = case.endswith("_split")
    case = case.replace("_split", "")
    if case == "vit":
        B, H, N, hd = 8, 12, 197, 64
    elif case == "mask_drop":
        B, H, N, hd = 5, 6, 150, 64
        p, seed = 0.1, 99
        key_pad = torch.zeros(B, N, dtype=torch.bool, device="cuda")
        key_pad[2, 120:] = True
        key_pad[4, 3] = True
    elif case == "hd128":
        B, H, N, hd = 4, 4, 100, 128
    elif case == "short":
        B, H, N, hd = 16, 8, 20, 96
    else:
        B, H, N, hd, dt = 3, 4, 77, 32, torch.float32
    D = H * hd
    qkv = torch.randn(B * N, 3 * D, device="cuda", generator=g).to(dt)
    do = torch.randn(B * N, D, device="cuda", generator=g).to(dt)
    o = torch.empty(B * N, D, device="cuda", dtype=dt)
    hv = lambda t, off, ld: HeadView(t, off, N * ld, ld)
    Q, K_, V_, O = hv(qkv, 0, 3 * D), hv(qkv, D, 3 * D), hv(qkv, 2 * D, 3 * D), hv(o, 0, D)
    sc = 1.0 / math.sqrt(hd)
    lse, kp = ops.attention_fwd(Q, K_, V_, O, B, H, N, N, hd, sc, key_pad=key_pad, drop=(p, seed))
    x = qkv.float().view(B, N, 3, H, hd)
    qr, kr, vr = (x[:, :, i].transpose(1, 2).contiguous().requires_grad_(True) for i in range(3))
    s = torch.einsum("bhqd,bhkd->bhqk", qr, kr) * sc
    if key_pad is not None:
        s = s.masked_fill(key_pad[:, None, None, :], float("-inf"))
    a = torch.softmax(s, -1)
    if p > 0:
        a = a * (ops.dropout_mask(B * H * N * N, p, seed).view(B, H, N, N).float() / (1 - p))
    torch.einsum("bhqk,bhkd->bhqd", a, vr).backward(do.float().view(B, N, H, hd).transpose(1, 2))
    ref = torch.cat([t.grad.sum((0, 2)).reshape(-1) for t in (qr, kr, vr)])  # [h, d] order = column h*hd + d
    dqkv = torch.empty_like(qkv)
    dbias = torch.full((3 * D,), 5.0, device="cuda")
    fused = hd == 64 and N > 32 and not split and dt == torch.bfloat16  # the attn_bwd_fused64 route
    try:
        if split:
            ops.check(L.capk_attention_set_fused_bwd(0), "set_fused_bwd")
        ops.attention_bwd_bias(Q, K_, V_, O, hv(do, 0, D), lse, hv(dqkv, 0, 3 * D), hv(dqkv, D, 3 * D),
                               hv(dqkv, 2 * D, 3 * D), B, H, N, N, hd, sc, dbias, key_pad_u8=kp, drop=(p, seed))
        plain = torch.empty_like(qkv)  # the same route without the bias sums
        ops.attention_bwd(Q, K_, V_, O, hv(do, 0, D), lse, hv(plain, 0, 3 * D), hv(plain, D, 3 * D),
                          hv(plain, 2 * D, 3 * D), B, H, N, N, hd, sc, key_pad_u8=kp, drop=(p, seed))
        acc = torch.full((3 * D,), 5.0, device="cuda")
        ops.attention_bwd_bias(Q, K_, V_, O, hv(do, 0, D), lse, hv(dqkv, 0, 3 * D), hv(dqkv, D, 3 * D),
                               hv(dqkv, 2 * D, 3 * D), B, H, N, N, hd, sc, acc, key_pad_u8=kp, drop=(p, seed),
                               accumulate=True)
    finally:
        L.capk_attention_set_fused_bwd(-1)
    tol = 1e-4 if dt == torch.float32 else 2e-2
    scale_ref = ref.abs().max()
    assert _rel(dbias, ref) < tol, _rel(dbias, ref)
    assert float((dbias[D:2 * D] - ref[D:2 * D]).abs().max()) < tol * float(scale_ref)  # analytically ~0
    own = dqkv.float().sum(0)  # column sums of the kernel's own (rounded) gradients
    assert _rel(dbias, own) < (1e-5 if dt == torch.float32 or fused else 1e-2), _rel(dbias, own)
    if fused or split:
        assert torch.equal(dqkv, plain)
    torch.testing.assert_close(acc, dbias + 5.0, rtol=0, atol=1e-4 * float(scale_ref) + 1e-5)


@cuda
def test_attention_bwd_batch_slices_identical(ops):
    """capk_attention_set_bwd_slice: the split backward alternating its dK/dV and dQ kernels over
    batch slices (the dropout mask index carries the slice's first image) gives bit-identical
    dQ / dK / dV to one launch pair over the whole batch -- ViT shape with a key-padding mask
    and probability dropout, slices that do and do not divide the batch."""
    from capk.ops import HeadView
    L = ops.lib()
    g = torch.Generator(device="cuda").manual_seed(41)
    B, H, N, hd, p, seed = 7, 4, 197, 64, 0.1, 1234
    D = H * hd
    qkv = torch.randn(B * N, 3 * D, device="cuda", generator=g).bfloat16()
    do = torch.randn(B * N, D, device="cuda", generator=g).bfloat16()
    o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
    key_pad = torch.zeros(B, N, dtype=torch.bool, device="cuda")
    key_pad[3, 150:] = True
    hv = lambda t, off, ld: HeadView(t, off, N * ld, ld)
    sc = 1.0 / math.sqrt(hd)
    lse, kp = ops.attention_fwd(hv(qkv, 0, 3 * D), hv(qkv, D, 3 * D), hv(qkv, 2 * D, 3 * D), hv(o, 0, D), B, H, N, N,
                                hd, sc, key_pad=key_pad, drop=(p, seed))
    outs = []
    try:
        for sl in (0, 2, 3, 7):
            ops.check(L.capk_attention_set_bwd_slice(sl), "set_bwd_slice")
            d = torch.full_like(qkv, float("nan"))
            ops.attention_bwd(hv(qkv, 0, 3 * D), hv(qkv, D, 3 * D), hv(qkv, 2 * D, 3 * D), hv(o, 0, D), hv(do, 0, D),
                              lse, hv(d, 0, 3 * D), hv(d, D, 3 * D), hv(d, 2 * D, 3 * D), B, H, N, N, hd, sc,
                              key_pad_u8=kp, drop=(p, seed))
            outs.append(d)
    finally:
        L.capk_attention_set_bwd_slice(-1)
    assert bool(torch.isfinite(outs[0].float()).all())
    for d in outs[1:]:
        assert torch.equal(d, outs[0])


@cuda
@pytest.mark.parametrize("case", ["vit", "pad_drop", "n100", "n256_gap"])
def test_attention_fused_bwd_matches_split(ops, case):
    """capk_attention_set_fused_bwd: the fused single-pass backward (one workgroup per (image,
    head), P and dS formed once) against the split dK/dV + dQ pair on the same inputs -- ViT
    shape, key padding + probability dropout, N = 100, N = 256 with a gap row between images.
    dK and dV come from the same per-key-block loop (identical); dQ sums the same bf16 dS
    blocks over the keys in the same order (rel. <= 5e-3), and both match fp32 autograd."""
    from capk.ops import HeadView
    L = ops.lib()
    g = torch.Generator(device="cuda").manual_seed(47)
    B, H, N, gap, p = {"vit": (12, 12, 197, 0, 0.0), "pad_drop": (9, 8, 197, 0, 0.1), "n100": (10, 4, 100, 0, 0.0),
                       "n256_gap": (6, 4, 256, 1, 0.0)}[case]
    hd = 64
    D = H * hd
    rows = (B - 1) * (N + gap) + N
    qkv = torch.randn(rows, 3 * D, device="cuda", generator=g).bfloat16()
    do = torch.randn(rows, D, device="cuda", generator=g).bfloat16()
    o = torch.empty(rows, D, device="cuda", dtype=torch.bfloat16)
    key_pad = None
    if case == "pad_drop":
        key_pad = torch.zeros(B, N, dtype=torch.bool, device="cuda")
        key_pad[3, 150:] = True
        key_pad[5, 7:12] = True
    hv = lambda t, off, ld: HeadView(t, off, (N + gap) * ld, ld)
    sc = 1.0 / math.sqrt(hd)
    drop = (p, 4321) if p > 0 else ops.NO_DROP
    lse, kp = ops.attention_fwd(hv(qkv, 0, 3 * D), hv(qkv, D, 3 * D), hv(qkv, 2 * D, 3 * D), hv(o, 0, D), B, H, N, N,
                                hd, sc, key_pad=key_pad, drop=drop)
    outs = []
    try:
        for mode in (0, 1):
            ops.check(L.capk_attention_set_fused_bwd(mode), "set_fused_bwd")
            d = torch.zeros_like(qkv)
            ops.attention_bwd(hv(qkv, 0, 3 * D), hv(qkv, D, 3 * D), hv(qkv, 2 * D, 3 * D), hv(o, 0, D), hv(do, 0, D),
                              lse, hv(d, 0, 3 * D), hv(d, D, 3 * D), hv(d, 2 * D, 3 * D), B, H, N, N, hd, sc,
                              key_pad_u8=kp, drop=drop)
            outs.append(d)
    finally:
        L.capk_attention_set_fused_bwd(-1)
    split, fused = outs
    assert bool(torch.isfinite(fused.float()).all())
    assert torch.equal(fused[:, D:], split[:, D:])  # dK, dV
    assert _rel(fused[:, :D], split[:, :D]) < 5e-3  # dQ
    if gap:
        gap_rows = torch.stack([fused[b * (N + gap) + N] for b in range(B - 1)])
        assert float(gap_rows.abs().max()) == 0.0
    if p == 0.0:  # vs fp32 autograd on the same bf16 values
        def heads(col0):
            t = torch.stack([qkv[b * (N + gap):b * (N + gap) + N, col0:col0 + D] for b in range(B)]).float()
            return t.view(B, N, H, hd).transpose(1, 2).requires_grad_(True)
        qr, kr, vr = heads(0), heads(D), heads(2 * D)
        ref = _attn_ref(qr, kr, vr, sc, False, key_pad)
        dor = torch.stack([do[b * (N + gap):b * (N + gap) + N] for b in range(B)]).float().view(B, N, H, hd).transpose(1, 2)
        ref.backward(dor)

        def got(col0):
            return torch.stack([fused[b * (N + gap):b * (N + gap) + N, col0:col0 + D] for b in range(B)]).float().view(
                B, N, H, hd).transpose(1, 2)
        assert _rel(got(0), qr.grad) < 3e-2
        assert _rel(got(D), kr.grad) < 3e-2
        assert _rel(got(2 * D), vr.grad) < 3e-2


@cuda
@pytest.mark.parametrize("nq,nk", [(200, 64), (40, 197), (256, 16), (250, 100), (197, 197), (64, 256)])
def test_attention_fused_bwd_ragged_after_poisoned_lds(ops, nq, nk):
    """The fused backward with Nq != Nk, at query counts past the workgroup's delta / lse passes
    of round 5 (Nq = 200 with 64 keys: 512 threads covered 128 queries), run right after every
    CU's LDS was filled with NaN (capk_debug_fill_lds) so a padded-row delta or lse the kernel did not write shows up as NaN.
    dK / dV equal the split pair's, dQ within 5e-3, all three vs fp32 autograd within 3e-2."""
    from capk.ops import HeadView
    L = ops.lib()
    g = torch.Generator(device="cuda").manual_seed(53)
    B, H, hd = 6, 4, 64
    D = H * hd
    q = torch.randn(B * nq, D, device="cuda", generator=g).bfloat16()
    kv = torch.randn(B * nk, 2 * D, device="cuda", generator=g).bfloat16()
    do = torch.randn(B * nq, D, device="cuda", generator=g).bfloat16()
    o = torch.empty(B * nq, D, device="cuda", dtype=torch.bfloat16)
    Q, K_, V_ = HeadView(q, 0, nq * D, D), HeadView(kv, 0, nk * 2 * D, 2 * D), HeadView(kv, D, nk * 2 * D, 2 * D)
    O, dO = HeadView(o, 0, nq * D, D), HeadView(do, 0, nq * D, D)
    sc = 1.0 / math.sqrt(hd)
    lse, _ = ops.attention_fwd(Q, K_, V_, O, B, H, nq, nk, hd, sc)
    outs = []
    try:
        for mode in (0, 1):
            ops.check(L.capk_attention_set_fused_bwd(mode), "set_fused_bwd")
            dq, dkv = torch.zeros_like(q), torch.zeros_like(kv)
            ops.check(L.capk_debug_fill_lds(0x7FC00000, ops._stream()), "debug_fill_lds")  # quiet NaN
            ops.attention_bwd(Q, K_, V_, O, dO, lse, HeadView(dq, 0, nq * D, D), HeadView(dkv, 0, nk * 2 * D, 2 * D),
                              HeadView(dkv, D, nk * 2 * D, 2 * D), B, H, nq, nk, hd, sc)
            outs.append((dq, dkv))
    finally:
        L.capk_attention_set_fused_bwd(-1)
    (dq_s, dkv_s), (dq_f, dkv_f) = outs
    assert bool(torch.isfinite(dq_f.float()).all()) and bool(torch.isfinite(dkv_f.float()).all())
    assert torch.equal(dkv_f, dkv_s)
    assert _rel(dq_f, dq_s) < 5e-3
    qr = q.float().view(B, nq, H, hd).transpose(1, 2).requires_grad_(True)
    kr = kv[:, :D].float().reshape(B, nk, H, hd).transpose(1, 2).detach().requires_grad_(True)
    vr = kv[:, D:].float().reshape(B, nk, H, hd).transpose(1, 2).detach().requires_grad_(True)
    _attn_ref(qr, kr, vr, sc, False, None).backward(do.float().view(B, nq, H, hd).transpose(1, 2))
    heads = lambda t, n: t.float().reshape(B, n, H, hd).transpose(1, 2)
    assert _rel(heads(dq_f, nq), qr.grad) < 3e-2
    assert _rel(heads(dkv_f[:, :D], nk), kr.grad) < 3e-2
    assert _rel(heads(dkv_f[:, D:], nk), vr.grad) < 3e-2


@cuda
def test_gemm_timer_follows_the_stream(ops):
    """bench.py's live GEMM timer (ops.GEMM_TIMER) records the GEMMs launched on the stream it
    was started on from any host thread -- those of a backward pass run on autograd's device
    thread -- and none launched on another stream (the config-5 baseline search's side stream)."""
    A = torch.randn(256, 256, device="cuda").bfloat16()
    C = torch.empty(256, 256, device="cuda", dtype=torch.bfloat16)

    def g():
        ops.gemm(A, True, A, True, 256, 256, 256, C, lda=256, ldb=256, ldc=256)

    class Fn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x * 2

        @staticmethod
        def backward(ctx, gy):
            g()
            return gy * 2

    x = torch.randn(8, device="cuda", requires_grad=True)
    side = torch.cuda.Stream()
    stride, ops.GEMM_TIMER.stride = ops.GEMM_TIMER.stride, 1  # bracket every launch
    ops.GEMM_TIMER.start()
    try:
        g()  # main stream, this thread
        Fn.apply(x).sum().backward()  # main stream, autograd's thread
        with torch.cuda.stream(side):
            g()  # another stream: not recorded
        side.synchronize()
    finally:
        ops.GEMM_TIMER.stop()
        ops.GEMM_TIMER.stride = stride
    assert ops.GEMM_TIMER.summary()["launches"] == 2
    ops.GEMM_TIMER.stride = 2  # sampling: launches 1, 3, 5 of 6 on the stream
    ops.GEMM_TIMER.start()
    try:
        for _ in range(6):
            g()
    finally:
        ops.GEMM_TIMER.stop()
        ops.GEMM_TIMER.stride = stride
    sm = ops.GEMM_TIMER.summary()
    assert sm["launches"] == 3 and sm["launches_seen"] == 6


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("M,K,N,conv", [(256, 768, 768, True), (256, 3072, 768, True), (1024, 3072, 768, True),
                                        (1280, 768, 768, False), (1280, 3072, 768, False), (40, 512, 512, False)])
def test_product_ln_slabs_bit_identical(M, K, N, conv):
    """ops.product_ln (split-K slabs summed by capk_layernorm_fwd_slabs) against the separate
    route (capk_gemm + bias + residual, then capk_layernorm_fwd), for the GPT-2 Conv1D [in, out]
    and nn.Linear [out, in] weights of the decode steps: LayerNorm output and the kept pre-LN sum
    bit-identical when both routes split K the same way (CAPK_SLAB_SPLITS=0, or shapes where the
    slab policy keeps capk_gemm's count), else within fp32 summation-order rounding of it (the
    slab route splits the short-K products further: no reduce launch to amortise); both vs an
    fp32 torch reference within 2e-2."""
    from capk import ops
    g = torch.Generator(device="cuda").manual_seed(M + K)
    bf = torch.bfloat16
    x = torch.randn(M, K, device="cuda", generator=g).to(bf)
    w = (torch.randn(K, N, device="cuda", generator=g) if conv else torch.randn(N, K, device="cuda", generator=g))
    w = (w / K ** 0.5).to(bf)
    b = torch.randn(N, device="cuda", generator=g)
    res = torch.randn(M, N, device="cuda", generator=g).to(bf)
    lw, lb = torch.rand(N, device="cuda", generator=g) + 0.5, torch.randn(N, device="cuda", generator=g)
    saved = ops.DECODE_SLABS
    try:
        ops.DECODE_SLABS = True
        y1, s1 = ops.product_ln(x, w, conv, b, res, lw, lb, 1e-5, keep=True)
        ops.DECODE_SLABS = False
        y0, s0 = ops.product_ln(x, w, conv, b, res, lw, lb, 1e-5, keep=True)
    finally:
        ops.DECODE_SLABS = saved
    import ctypes
    sp = ctypes.c_int(0)
    ops.lib().capk_gemm_slabs_workspace(M, N, K, ctypes.byref(sp))
    if sp.value == 1:  # (then capk_gemm's own count is 1 as well: the slab policy only raises it)
        assert torch.equal(s1, s0)
        assert torch.equal(y1, y0)
    else:
        assert float((s1.float() - s0.float()).norm() / s0.float().norm()) < 1e-2
        assert float((y1.float() - y0.float()).norm() / y0.float().norm()) < 1e-2
    ref = torch.nn.functional.layer_norm((x.float() @ (w.float() if conv else w.float().t())) + b + res.float(),
                                         (N,), lw, lb, 1e-5)
    assert float((y1.float() - ref).norm() / ref.norm()) < 2e-2


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_zero_gap_rows():
    """capk_zero_gap_rows clears exactly rows b * rpb + j (S <= j < rpb) of a strided per-image
    buffer -- the decoder's cross-attention K / V gradient over the ViT sequence minus its CLS
    rows (M_ext = (B - 1) rpb + S rows, so the last image has no gap row) -- and nothing else."""
    from capk import ops
    B, rpb, S, C = 7, 197, 196, 1536
    M = (B - 1) * rpb + S
    x = torch.randn(M, C, device="cuda").bfloat16()
    ref = x.clone()
    for b in range(B):
        for j in range(S, rpb):
            r = b * rpb + j
            if r < M:
                ref[r] = 0
    ops.zero_gap_rows(x, B, rpb, S)
    assert torch.equal(x, ref)
